"""Model registry with the reference's names (main.py:32-56, subset on the
hot path: 'lgn' = LightGCN, 'mf' = MF, 'sage' = GraphSAGE, 'sasrec' = SASRec)."""
from .graphsage import GraphSAGE
from .lightgcn import LightGCN
from .mf import MF
from .sasrec import SASRec

MODELS = {
    "mf": MF,
    "lgn": LightGCN,
    "sage": GraphSAGE,
    "sasrec": SASRec,
}
