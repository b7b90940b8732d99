import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "furusato_recommend_amd", "libmirec.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    if not os.path.exists(LIB):
        # Cross-compiles for gfx950; works without a GPU.
        subprocess.run(["make", "-C", os.path.join(ROOT, "furusato_recommend_amd", "csrc"),
                        "-j8"], check=True, stdout=subprocess.DEVNULL)


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
    return load
