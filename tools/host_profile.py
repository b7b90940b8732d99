"""Host-side cost of a training step (cProfile over K steps after warmup):
where the Python / dispatch time of a host-bound step goes.

    python tools/host_profile.py c4 [--steps K]     # SASRec (C4)
    python tools/host_profile.py c3 [--steps K]     # GraphSAGE (C3)
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def c4_step_fn(B=2048):
    from furusato_recommend_amd import SASRec
    from furusato_recommend_amd.sasrec import SequenceData

    class DS:
        n_users, m_items = 1_000_000, 100_000
    dev = torch.device("cuda:0")
    seq = SequenceData.synthetic(DS.n_users, DS.m_items, dev, max_len=50, min_len=5, seed=0)
    m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                "device": "cuda:0", "bpr_batch_size": B, "dropout_p": 0.2}, DS, sequences=seq)
    rng = np.random.default_rng(7)
    g = torch.Generator(device=dev).manual_seed(7)

    def step():
        u_h = rng.integers(0, DS.n_users, B)
        u = m._upload(u_h)
        k = (torch.rand(B, device=dev, generator=g) * seq.length[u]).long()
        p = seq.items[u, k].long()
        n = torch.randint(0, DS.m_items, (B,), device=dev, generator=g)
        m.stageOne(u_h, p, n)
    return step


def c3_step_fn(B=2048):
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    torch.manual_seed(2020)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3, "decay": 1e-7,
                   "device": "cuda:0", "bpr_batch_size": B}, ds)
    it = [0]

    def step():
        u, p, n = m.sample(B, seed=7, offset=it[0] * B)
        it[0] += 1
        m.stageOne(u, p, n)
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["c3", "c4"])
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    step = c4_step_fn() if args.which == "c4" else c3_step_fn()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"host enqueue {1e3 * t_host / args.steps:.3f} ms/step, "
          f"wall {1e3 * t_all / args.steps:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
    print(s.getvalue())


if __name__ == "__main__":
    main()
