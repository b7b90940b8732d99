"""furusato_recommend_amd — MI355X-native LightGCN propagation + BPR engine.

Drop-in for the training hot path of HiromasaYamanishi/furusato_recommend
(model/lgcn.py, model/MF.py, negative_sample.py, ddp_lgcn.py) built on
libmirec.so, a C-ABI library of hand-written gfx950 HIP kernels
(include/mirec.h).  Importing the package loads the library; there is no
CPU fallback.
"""
from ._lib import LIB_PATH, MirecError  # noqa: F401  (fails loudly if not built)
from .dataloader import FiveCore, Loader, SyntheticBipartite  # noqa: F401
from .graph import Graph  # noqa: F401
from .graphsage import GraphSAGE  # noqa: F401
from .lgconv import LGConv  # noqa: F401
from . import ops  # noqa: F401  (registers torch.ops.mirec.*)
from .lightgcn import LightGCN  # noqa: F401
from .mf import MF  # noqa: F401
from .sasrec import SASRec  # noqa: F401
from .register import MODELS  # noqa: F401

__all__ = ["LGConv", "LightGCN", "MF", "GraphSAGE", "SASRec", "Graph", "Loader", "SyntheticBipartite", "FiveCore", "MODELS",
           "MirecError", "LIB_PATH"]
