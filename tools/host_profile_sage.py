"""Host-side (Python) profile of the C3 GraphSAGE step: cProfile over K
steps of GraphSAGE.stageOne, optionally as C micro-batches (the pipelined
exchange's shape, with a no-op chunk hook), top functions by own time.
Where the host spends the time it needs to issue one step's launches.

    python tools/host_profile_sage.py [--chunks C] [--steps K]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--bwd-main-thread", type=int, default=0,
                    help="1: the autograd backward on the calling thread (visible to cProfile)")
    args = ap.parse_args()
    if args.bwd_main_thread:
        torch.autograd.set_multithreading_enabled(False)
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    dev = torch.device("cuda:0")
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    torch.manual_seed(2020)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3, "decay": 1e-7,
                   "device": str(dev), "bpr_batch_size": 2048}, ds)
    C = args.chunks
    kw = {}
    if C > 1:
        def chunk_hook(k, phase):
            if phase == "post":
                m._tg.pending = True  # the step's Adam consumes the last one
        kw = {"chunks": C, "chunk_hook": chunk_hook}
    step_no = [0]

    def step():
        u, p, n = m.sample(2048, seed=7, offset=step_no[0] * 2048)
        step_no[0] += 1
        m.stageOne(u, p, n, **kw)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps * 1e3
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(args.steps):
        step()
    pr.disable()
    host = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize()
    print(f"chunks={C} wall {wall:.3f} ms/step; host issue under cProfile {host:.3f} ms/step")
    pstats.Stats(pr).sort_stats("tottime").print_stats(args.top)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
