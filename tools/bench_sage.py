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


def cpu_baseline(m, B, fan, k=3):
    """The oracle's restatement of graphsage.py:311-337 (torch CPU fp32) on
    the same workload, timed per BASELINE.md §3: one warm-up training step,
    then the mean of ``k`` steps, each on its own sampled tree (drawn by the
    GPU sampler, copied to the host): forward, loss with the reference's
    parameter norms, backward, torch Adam over every parameter."""
    import bench
    from oracle import lightgcn_oracle as O
    threads = bench.host_threads()
    torch.set_num_threads(threads)
    table = m._table.detach().cpu().clone().requires_grad_(True)
    lin = [torch.nn.Linear(2 * m.latent_dim, m.latent_dim) for _ in m.w_linears]
    for a, b in zip(lin, m.w_linears):
        a.load_state_dict({kk: v.detach().cpu() for kk, v in b.state_dict().items()})
    params = [table] + [q for layer in lin for q in layer.parameters()]
    opt = torch.optim.Adam(params, lr=1e-3)
    times, rows = [], 0
    for i in range(k + 1):
        u, p, n = m.sample(B, seed=99, offset=i * B)
        seeds = torch.cat([u, p + m.n_user, n + m.n_user])
        groups = [g.cpu().numpy() for g, _ in m.sample_tree(seeds, 12345 + i).groups]
        rows = sum(g.size for g in groups)
        t0 = time.perf_counter()
        opt.zero_grad()
        emb = O.sage_forward(table, lin, groups, m.num_layers, m.sizes)
        ue, pe, ne = emb[:B], emb[B:2 * B], emb[2 * B:]
        reg = [table[:m.n_user], table[m.n_user:]] + [q for layer in lin
                                                      for q in (layer.weight, layer.bias)]
        loss = O.sage_loss(ue, pe, ne, reg, 1e-7)
        loss.backward()
        opt.step()
        if i:  # i = 0 is the warm-up
            times.append(time.perf_counter() - t0)
    t = sum(times) / len(times)
    return {"value": round(B / t, 2), "unit": "positive-edges/s", "cores": threads,
            "threads": threads, "os_cpu_count": os.cpu_count(), "kind": "port",
            "cpu": bench.cpu_model(), "warmup": 1, "k": k, "step_s": round(t, 3),
            "step_s_each": [round(x, 3) for x in times],
            "sample": f"1 warm-up + mean of {k} training steps (B={B}, fanout {fan}) of the C3 "
                      f"workload, each on its own sampled tree (~{rows} rows), dense Adam over "
                      f"the id table"}


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
    ap.add_argument("--table-exchange", choices=("auto", "fetch", "routed", "dense"), default="auto",
                    help="data-parallel exchange of the id table (dist.DenseGradDataParallel)")
    ap.add_argument("--rehearse", action="store_true",
                    help="all ranks on cuda:0, gloo collectives (N-rank path on one GPU)")
    args = ap.parse_args()
    if args.steps < 1:
        ap.error("--steps must be >= 1")
    from furusato_recommend_amd import graphsage as _gs
    _gs.SORTED_LEAF_BACKWARD = args.leaf_bwd == "sorted"
    if args.blas:
        torch.backends.cuda.preferred_blas_library(args.blas)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = 0 if args.rehearse else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        from furusato_recommend_amd.dist import init_distributed
        init_distributed("gloo" if args.rehearse else "nccl", dev)
    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    from furusato_recommend_amd.dist import DenseGradDataParallel
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0, kind=args.kind)
    torch.manual_seed(2020)
    fan = [int(x) for x in args.fanouts.split(",")]
    m = GraphSAGE({"recdim": args.dim, "layer": len(fan), "fanouts": fan, "lr": 1e-3,
                   "decay": 1e-7, "device": str(dev), "bpr_batch_size": args.batch}, ds)
    dp = DenseGradDataParallel(m, table_exchange=None if args.table_exchange == "auto"
                               else args.table_exchange)
    B = args.batch

    def step(i):
        u, p, n = m.sample(B, seed=7, offset=i * B, shard=rank, n_shards=world)
        dp.step(u, p, n)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    tg = m._tg
    # HIP events (the dominant kernel, timed live; the collectives) on every
    # 4th timed step only: each event record idles the GPU ~5 us (bench.py)
    comm_ev, adam_ev, sampled = [], [], 0
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for j, i in enumerate(range(args.warmup, args.warmup + args.steps)):
        on = j % 4 == 3 or (args.steps < 4 and j == args.steps - 1)
        sampled += int(on)
        dp.comm_events = comm_ev if (on and world > 1) else None
        tg.adam_events = adam_ev if (on and world == 1) else None
        step(i)
    torch.cuda.synchronize()
    dp.comm_events = comm_ev if world > 1 else None
    tg.adam_events = adam_ev if world == 1 else None
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    comm = None
    if world > 1:
        from furusato_recommend_amd.dist import _elapsed_ms
        cm = _elapsed_ms(dp.comm_events) / sampled
        t = torch.tensor([cm], dtype=torch.float64, device="cpu" if args.rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cm = float(t.item())
        comm = {"backend": dist.get_backend(), "world_size": world,
                "table_exchange": dp.table_exchange, "comm_ms_per_step": round(cm, 4),
                "exchange_bytes_per_rank": dp.last_exchange_bytes,
                "exchange_bytes_note": "bytes rank 0 received in the last step",
                "algbw_GBps": round(dp.last_exchange_bytes / (cm * 1e-3) / 1e9, 2) if cm else None}
    roof = None
    if tg.adam_events:
        # tg_adam_kernel (+ its 2-float norm finalize in the same bracket):
        # W, m, v read and written, the stamps, and the tree-sum rows of the
        # last step (stamp == gen) read — per launch
        ms = sum(a.elapsed_time(b) for a, b in tg.adam_events) / len(tg.adam_events)
        touched = int((tg.stamp == tg.gen).sum())
        nbytes = 6 * tg.n_rows * tg.dim * 4 + tg.n_rows * 4 + touched * tg.dim * 4
        roof = {"bound": "hbm", "kernel": "tg_adam_kernel (fused table Adam)",
                "achieved": round(nbytes / (ms * 1e-3) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(nbytes / (ms * 1e-3) / 1e9 / 8000.0, 4),
                "traffic": 3660651465, "traffic_source": "profiles/round6_final_pmc_tg_adam.json",
                "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": nbytes,
                "launches_per_step": round(len(tg.adam_events) / sampled, 2),
                "timed_steps_sampled": sampled}
        tg.adam_events = None
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline(m, B, fan)
    if rank == 0:
        print(json.dumps({
            "metric": "GraphSAGE BPR positive-edges/sec (C3)", "value": round(world * args.steps * B / dt, 1),
            "unit": "positive-edges/s", "n_gpus": world, "steps": args.steps,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "dtype": "f32",
            "gemm_arith": "f32 products as an exact three-term bf16 split on bf16 MFMA (f32-class error: DESIGN.md section 4, profiles/round3c_gemm_split_accuracy.jsonl)",
            "config": {"workload": "C3: GraphSAGE 2-hop fanout %s d=%d on the C2 graph" % (fan, args.dim)
                        + ("" if args.kind == "uniform" else " (%s item popularity)" % args.kind),
                       "bpr_batch_per_rank": B,
                       "parallelism": (f"dp{world} rehearsal (gloo, one GPU)" if args.rehearse
                                       else f"dp{world} (user-sharded, {dp.table_exchange} "
                                            f"table exchange)"),
                       "leaf_bwd": args.leaf_bwd},
            "roofline": roof,
            "comm": comm,
            "cpu_baseline": cpu}),
            flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
