"""Probe: can the SASRec (C4) training step be captured in a HIP graph, and
what does a replay cost against the eager step?  Replays one fixed batch
(the seeds / Adam scalars baked in at capture: timing only, not training).

    python tools/graph_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from furusato_recommend_amd import SASRec
    from furusato_recommend_amd.sasrec import SequenceData

    class DS:
        n_users, m_items = 1_000_000, 100_000
    B = 2048
    dev = torch.device("cuda:0")
    seq = SequenceData.synthetic(DS.n_users, DS.m_items, dev, max_len=50, min_len=5, seed=0)
    m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                "device": "cuda:0", "bpr_batch_size": B, "dropout_p": 0.2,
                "attn_buckets": False}, DS, sequences=seq)
    rng = np.random.default_rng(7)
    u_h = rng.integers(0, DS.n_users, B)
    u = torch.as_tensor(u_h, device=dev)
    p = seq.items[u, 0].long()
    n = torch.randint(0, DS.m_items, (B,), device=dev)

    def eager():
        return m.stageOne(u_h, p, n)

    # the staging upload (pinned copy + event wait) stays outside a graph
    from furusato_recommend_amd.sasrec import length_buckets
    up_static = torch.as_tensor(np.concatenate([u_h, length_buckets(seq.length_host[u_h])[0]]),
                                device=dev)
    m._upload = lambda host_ids: up_static

    for _ in range(5):
        eager()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        eager()
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / 30

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            eager()
    torch.cuda.current_stream().wait_stream(s)
    for q in m.parameters():
        q.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_loss = eager()
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        g.replay()
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / 30
    print(f"eager {1e3 * t_eager:.3f} ms/step, graph replay {1e3 * t_graph:.3f} ms/step, "
          f"loss {float(static_loss):.4f}", flush=True)


if __name__ == "__main__":
    main()
