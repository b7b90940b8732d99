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


def cpu_baseline(m, B, fan):
    """The oracle's restatement of graphsage.py:311-337 (torch CPU fp32) on
    one batch of the same workload: one sampled tree
    (drawn by the GPU sampler, copied to the host), forward, loss with the
    reference's parameter norms, backward, torch Adam over every parameter."""
    import platform

    from oracle import lightgcn_oracle as O
    # torch's default intra-op pool (OMP_NUM_THREADS: 16 on the GPU box), as
    # bench.py's baseline
    u, p, n = m.sample(B, seed=99, offset=0)
    seeds = torch.cat([u, p + m.n_user, n + m.n_user])
    tree = m.sample_tree(seeds, 12345)
    groups = [g.cpu().numpy() for g, _ in tree.groups]
    table = m._table.detach().cpu().clone().requires_grad_(True)
    lin = [torch.nn.Linear(2 * m.latent_dim, m.latent_dim) for _ in m.w_linears]
    for a, b in zip(lin, m.w_linears):
        a.load_state_dict({k: v.detach().cpu() for k, v in b.state_dict().items()})
    params = [table] + [q for layer in lin for q in layer.parameters()]
    opt = torch.optim.Adam(params, lr=1e-3)
    t0 = time.perf_counter()
    emb = O.sage_forward(table, lin, groups, m.num_layers, m.sizes)
    ue, pe, ne = emb[:B], emb[B:2 * B], emb[2 * B:]
    reg = [table[:m.n_user], table[m.n_user:]] + [q for layer in lin for q in (layer.weight,
                                                                              layer.bias)]
    loss = O.sage_loss(ue, pe, ne, reg, 1e-7)
    loss.backward()
    opt.step()
    t = time.perf_counter() - t0
    cpu_name = platform.processor() or "cpu"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_name = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": round(B / t, 2), "unit": "positive-edges/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu": cpu_name, "step_s": round(t, 3),
            "sample": f"1 training step (B={B}, fanout {fan}) of the C3 workload: tree of "
                      f"{sum(g.size for g in groups)} rows, dense Adam over the id table"}


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
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--kind", choices=("uniform", "zipf"), default="uniform",
                    help="synthetic graph: uniform (C3) or Zipf item popularity (hub rows)")
    ap.add_argument("--blas", default="", help="torch BLAS backend override (cublas / cublaslt)")
    ap.add_argument("--leaf-bwd", choices=("sorted", "atomic"), default="sorted",
                    help="leaf-hop backward: radix-sorted ordered sums or float atomics")
    args = ap.parse_args()
    from furusato_recommend_amd import graphsage as _gs
    _gs.SORTED_LEAF_BACKWARD = args.leaf_bwd == "sorted"
    if args.blas:
        torch.backends.cuda.preferred_blas_library(args.blas)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    from furusato_recommend_amd.dist import DenseGradDataParallel
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0, kind=args.kind)
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
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline(m, B, fan)
    if rank == 0:
        print(json.dumps({
            "metric": "GraphSAGE BPR positive-edges/sec (C3)", "value": round(world * args.steps * B / dt, 1),
            "unit": "positive-edges/s", "n_gpus": world, "steps": args.steps,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "dtype": "f32",
            "config": {"workload": "C3: GraphSAGE 2-hop fanout %s d=%d on the C2 graph" % (fan, args.dim)
                        + ("" if args.kind == "uniform" else " (%s item popularity)" % args.kind),
                       "bpr_batch_per_rank": B, "parallelism": f"dp{world} (dense grad all-reduce)",
                       "leaf_bwd": args.leaf_bwd},
            "cpu_baseline": cpu}),
            flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
