"""Config C3 (BASELINE.json configs[2]): GraphSAGE 2-hop fanout [25,10]
d=128 on the C2 synthetic graph (1M users x 100K items / 20M edges), user-
sharded data parallelism.  Prints one JSON line (positive-edges/s).

    python tools/bench_sage.py [--steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N tools/bench_sage.py
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--fanouts", default="25,10")
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    from furusato_recommend_amd.dist import DenseGradDataParallel
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0)
    torch.manual_seed(2020)
    fan = [int(x) for x in args.fanouts.split(",")]
    m = GraphSAGE({"recdim": args.dim, "layer": len(fan), "fanouts": fan, "lr": 1e-3,
                   "decay": 1e-7, "device": str(dev), "bpr_batch_size": args.batch}, ds)
    dp = DenseGradDataParallel(m)
    B = args.batch

    def step(i):
        u, p, n = m.sample(B, seed=7, offset=i * B, shard=rank, n_shards=world)
        dp.step(u, p, n)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({
            "metric": "GraphSAGE BPR positive-edges/sec (C3)", "value": round(world * args.steps * B / dt, 1),
            "unit": "positive-edges/s", "n_gpus": world, "steps": args.steps,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "dtype": "f32",
            "config": {"workload": "C3: GraphSAGE 2-hop fanout %s d=%d on the C2 graph" % (fan, args.dim),
                       "bpr_batch_per_rank": B, "parallelism": f"dp{world} (dense grad all-reduce)"}}),
            flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
