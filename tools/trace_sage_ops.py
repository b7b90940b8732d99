"""Debug helper: which aten ops (and shapes) a GraphSAGE step launches."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3, "decay": 1e-7,
                   "device": "cuda:0", "bpr_batch_size": 2048}, ds)
    for i in range(3):
        m.stageOne(*m.sample(2048, seed=7, offset=i * 2048))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        m.stageOne(*m.sample(2048, seed=7, offset=99 * 2048))
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=40,
                                                            max_name_column_width=40,
                                                            max_shapes_column_width=90))


if __name__ == "__main__":
    main()
