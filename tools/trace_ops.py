"""Debug helper: host-side (CPU) cost of one training step by aten op and
autograd node, for the SASRec (C4) or GraphSAGE (C3) model."""
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "sasrec"
    dev = torch.device("cuda:0")
    if which == "sasrec":
        from furusato_recommend_amd import SASRec
        from furusato_recommend_amd.sasrec import SequenceData

        class DS:
            n_users, m_items = 1_000_000, 100_000
        seq = SequenceData.synthetic(1_000_000, 100_000, dev, max_len=50, seed=0)
        m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                    "device": "cuda:0", "bpr_batch_size": 2048, "dropout_p": 0.2}, DS(),
                   sequences=seq)
        rng = np.random.default_rng(0)

        def step():
            u = rng.integers(0, 1_000_000, 2048)
            p = torch.randint(0, 100_000, (2048,), device=dev)
            n = torch.randint(0, 100_000, (2048,), device=dev)
            m.stageOne(u, p, n)
    else:
        from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
        ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
        m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3,
                       "decay": 1e-7, "device": "cuda:0", "bpr_batch_size": 2048}, ds)

        def step():
            m.stageOne(*m.sample(2048, seed=7, offset=0))
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30,
                                    max_name_column_width=55))


if __name__ == "__main__":
    main()
