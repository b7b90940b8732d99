"""What micro-batching costs the C3 step on one GPU, with no exchange: the
GraphSAGE step (C3 config) as one batch and as C micro-batches
(GraphSAGE.stageOne(chunks=C), hooks that do nothing — the pipelined fetch
exchange's local step minus its exchange work), timed alternately.  The
difference is the part of the W = 8 rank step of tools/bench_world_sim.py
that micro-batching itself adds.  Timing only (with no export hook the
micro-batches' table gradients are not kept).  One JSON line per timing.

    python tools/sage_chunks.py [--chunks 1,2,3] [--steps 30] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="1,2,3")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    dev = torch.device("cuda:0")
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    torch.manual_seed(2020)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3, "decay": 1e-7,
                   "device": str(dev), "bpr_batch_size": a.batch}, ds)
    B = a.batch
    nxt = [0]

    def step(C):
        u, p, n = m.sample(B, seed=7, offset=nxt[0] * B)
        nxt[0] += 1
        if C == 1:
            m.stageOne(u, p, n)
        else:
            m.stageOne(u, p, n, chunks=C, chunk_hook=lambda k, phase: None)

    for r in range(a.rounds):
        for C in [int(c) for c in a.chunks.split(",")]:
            for _ in range(a.warmup):
                step(C)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(C)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            print(json.dumps({"round": r, "chunks": C, "ms_per_step": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
