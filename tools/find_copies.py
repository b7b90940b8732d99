"""Debug: which ops of the eager SASRec (C4) step issue device-to-device
copies (aten::copy_ / clone -> hipMemcpyAsync = __amd_rocclr_copyBuffer in
the captured graph): shapes and the Python call sites."""
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    dev = torch.device("cuda:0")
    from furusato_recommend_amd import SASRec
    from furusato_recommend_amd.sasrec import SequenceData

    class DS:
        n_users, m_items = 1_000_000, 100_000
    seq = SequenceData.synthetic(1_000_000, 100_000, dev, max_len=50, seed=0)
    m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                "device": "cuda:0", "bpr_batch_size": 2048, "dropout_p": 0.2, "graph": False},
               DS(), sequences=seq)
    rng = np.random.default_rng(0)

    def step():
        u = rng.integers(0, 1_000_000, 2048)
        p = torch.randint(0, 100_000, (2048,), device=dev)
        n = torch.randint(0, 100_000, (2048,), device=dev)
        m.stageOne(u, p, n)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::_to_copy"):
            stack = [s for s in (ev.stack or []) if "furusato_recommend_amd" in s or "torch/autograd" in s]
            print(ev.name, ev.input_shapes[:2], " | ".join(stack[:3]))


if __name__ == "__main__":
    main()
