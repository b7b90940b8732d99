"""Debug helper: which Python lines launch the non-mirec kernels (torch
elementwise ops, fills, copies) of one C3 (GraphSAGE) or C4 (SASRec, eager:
no graph capture) training step — torch profiler with CUDA activity, ops
grouped by their Python stack."""
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(which, dev):
    if which == "sasrec":
        from furusato_recommend_amd import SASRec
        from furusato_recommend_amd.sasrec import SequenceData

        class DS:
            n_users, m_items = 1_000_000, 100_000
        seq = SequenceData.synthetic(1_000_000, 100_000, dev, max_len=50, seed=0)
        m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                    "device": "cuda:0", "bpr_batch_size": 2048, "dropout_p": 0.2,
                    "graph": False}, DS(), sequences=seq)
        rng = np.random.default_rng(0)

        def step():
            u = rng.integers(0, 1_000_000, 2048)
            p = torch.randint(0, 100_000, (2048,), device=dev)
            n = torch.randint(0, 100_000, (2048,), device=dev)
            m.stageOne(u, p, n)
        return step
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3,
                   "decay": 1e-7, "device": "cuda:0", "bpr_batch_size": 2048}, ds)

    def step():
        m.stageOne(*m.sample(2048, seed=7, offset=0))
    return step


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "sage"
    dev = torch.device("cuda:0")
    step = build(which, dev)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 with_stack=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    rows = prof.key_averages(group_by_stack_n=6)
    keep = [e for e in rows if e.key.startswith("aten::") and e.self_device_time_total > 0]
    keep.sort(key=lambda e: -e.self_device_time_total)
    for e in keep[:25]:
        print(f"{e.key:32s} calls={e.count:4d} dev_us={e.self_device_time_total:9.1f}")
        for s in e.stack[:6]:
            if "site-packages" not in s:
                print("      ", s)
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25,
                                    max_name_column_width=70))


if __name__ == "__main__":
    main()
