"""Headline benchmark: BPR positive-edges/sec (+ Recall@20) for LightGCN-3
d=64 on the synthetic 1M users x 100K items / 20M-edge graph (BASELINE.json
configs[1]), 1..8 MI355X, user-sharded data parallelism over RCCL.

A step = draw B triples on device (each rank from its user shard) + one
training step (3-layer forward, fused BPR, 3-layer backward, Adam over the
whole table) — the reference's UniformSample + stageOne
(negative_sample.py:98-134, model/lgcn.py:127-133).  With --prune 1
(default) the layers the loss reads only on the batch's frontier are
computed there only (engine.py); --prune 0 runs every layer on every row.  `value` = triples
consumed by all ranks / wall time of the K timed steps (max over ranks),
inputs resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# mirec::prop_kernel<D=64, UNROLL=4, IN_PRESCALED, in_mask=false, row_mask=false>
DOMINANT = "prop_kernel<D, UNROLL, 0, false, false>"
KIND_NAMES = {0: "prescaled", 1: "raw", 2: "sparse", 3: "none"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048, help="bpr_batch_size per rank (parse.py:6)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--kind", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--cpu-baseline", default="step", choices=["step", "forward", "off"])
    ap.add_argument("--recall", type=int, default=1)
    ap.add_argument("--seed", type=int, default=2020)
    ap.add_argument("--prune", type=int, default=1,
                    help="frontier pruning (1) or every layer on every row (0)")
    ap.add_argument("--dp-mode", default="sparse", choices=["sparse", "dense"])
    return ap.parse_args()


def c2_workload(args) -> bool:
    return (args.users, args.items, args.edges) == (1_000_000, 100_000, 20_000_000)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(ds, args, users, pos, neg):
    """The CPU oracle (torch, fp32, all host threads given to torch) on a
    bounded sample of the same workload: one full training step (B triples)
    on the full C2 graph, or the 3-layer forward only."""
    from oracle.lightgcn_oracle import OracleLightGCN, forward
    threads = torch.get_num_threads()
    o = OracleLightGCN(ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, args.dim,
                       args.layers, 1e-3, 1e-4, seed=args.seed)
    t0 = time.perf_counter()
    with torch.no_grad():
        forward(o.emb, o.ei, ds.n_users, args.layers, o.div)
    t_fwd = time.perf_counter() - t0
    res = {"cores": threads, "kind": "port", "cpu": cpu_model(),
           "forward_s": round(t_fwd, 3)}
    if args.cpu_baseline == "step":
        t0 = time.perf_counter()
        o.stageOne(users, pos, neg)
        t_step = time.perf_counter() - t0
        res.update(value=round(len(users) / t_step, 3), unit="positive-edges/s",
                   step_s=round(t_step, 3),
                   sample=f"1 full training step (B={len(users)}) of the C2 workload "
                          f"(3-layer fwd+bwd+Adam over {ds.n_users + ds.m_items} nodes, "
                          f"{2 * ds.trainDataSize} adjacency entries)")
    else:
        res.update(value=round(1.0 / t_fwd, 4), unit="forward passes/s",
                   sample="one 3-layer full-graph forward of the C2 graph")
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.dist import DataParallel
    from furusato_recommend_amd.engine import sample_triples

    t_setup = time.perf_counter()
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0, kind=args.kind)
    torch.manual_seed(args.seed)
    cfg = {"recdim": args.dim, "layer": args.layers, "lr": 1e-3, "decay": 1e-4,
           "device": str(dev), "bpr_batch_size": args.batch, "prune": bool(args.prune)}
    model = LightGCN(cfg, ds)
    eng = model.engine
    emb = model.all_embedding.weight.data
    dp = DataParallel(eng, emb, model.optim, mode=args.dp_mode) if world > 1 else None
    B = args.batch
    u = torch.empty(B, dtype=torch.int32, device=dev)
    p, n = torch.empty_like(u), torch.empty_like(u)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup

    def step(i):
        sample_triples(model.graph, B, args.seed, i * B, u, p, n, err, rank, world)
        if dp is None:
            eng.train_step(emb, model.optim, u, p, n, cfg["decay"])
        else:
            dp.step(u, p, n, cfg["decay"])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    eng.prop_events = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    events, eng.prop_events = eng.prop_events, None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if int(err.item()) != 0:
        raise RuntimeError("sampler retry budget exhausted")

    # Live per-launch timing of the propagation kernel (HIP events on the
    # stream it is launched on), by launch kind (in_mode, in_mask, row_mask).
    # The roofline is quoted for the full (unmasked) pre-scaled launches,
    # whose algorithmic bytes are exact; masked launches touch data-dependent
    # subsets and are reported by time only.
    # A launch with an out_mask (forward layer 1 under pruning: layer sum
    # kept on F1 only) moves 2·|F1|·D·4 more bytes than launch_bytes counts;
    # |F1| is taken from the last step's mask (it varies by <0.5 % per step).
    f1_rows = int((eng.bm_hop.view(torch.uint8)[: model.graph.n_nodes] != 0).sum())
    per_kind = {}
    for s, e, kind, nbytes in events:
        ms = s.elapsed_time(e)
        if kind[3]:
            nbytes += 2 * f1_rows * args.dim * 4
        key = kind[:3]  # one rocprof kernel per (mode, in_mask, row_mask)
        d = per_kind.setdefault(key, [0, 0.0, 0])
        d[0] += 1
        d[1] += ms
        d[2] += nbytes
    t_prop = sum(v[1] for v in per_kind.values()) / args.steps
    dom = per_kind.get((0, False, False), [1, 1.0, 0])
    avg_ms = dom[1] / dom[0]
    avg_bytes = dom[2] / dom[0]
    achieved = avg_bytes / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_prop_kernel.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            j = json.load(f)
        kname = f"prop_kernel<{args.dim}, {({32: 2, 64: 4, 128: 4, 256: 8}).get(args.dim, 1)}, 0, false, false>"
        if (c2_workload(args) and j.get("workload") == f"C2-{args.kind}-d{args.dim}-L{args.layers}"
                and kname in j.get("kernel", "")):
            traffic = j.get("hbm_bytes_per_launch")

    recall = None
    if args.recall and rank == 0:
        from furusato_recommend_amd.evaluate import evaluate
        r = evaluate(model, ds.testDict, topks=(10, 20))
        recall = {"recall@20": float(r["recall"][1]), "ndcg@20": float(r["ndcg"][1]),
                  "recall@10": float(r["recall"][0]), "test_users": len(ds.testDict)}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        cpu = cpu_baseline(ds, args, u.cpu().numpy(), p.cpu().numpy(), n.cpu().numpy())

    if rank == 0:
        value = world * args.steps * B / dt
        c2 = (args.users, args.items, args.edges, args.dim, args.layers) == \
            (1_000_000, 100_000, 20_000_000, 64, 3)
        wl = ("C2" if c2 else "custom") + (
            f": LightGCN {args.layers}-layer d={args.dim}, synthetic {args.users} users x "
            f"{args.items} items / {args.edges} edges ({args.kind})")
        line = {
            "metric": f"BPR positive-edges/sec (LightGCN-{args.layers} d={args.dim}, "
                      f"{args.users} x {args.items} / {args.edges} edges)",
            "value": round(value, 1),
            "unit": "positive-edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY §8d C2 recipe, seed 0), random-init N(0, 0.1) weights",
            "config": {"workload": wl,
                       "users": args.users, "items": args.items, "edges": args.edges,
                       "graph": args.kind, "dim": args.dim, "layers": args.layers,
                       "bpr_batch_per_rank": B, "global_batch": B * world,
                       "parallelism": f"dp{world} (user-sharded, RCCL {args.dp_mode} "
                                      f"gradient exchange)"},
            "roofline": {"bound": "hbm",
                         "kernel": DOMINANT.replace("D, UNROLL", f"{args.dim}, "
                                                    f"{ {32: 2, 64: 4, 128: 4, 256: 8}.get(args.dim, 1)}"),
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "avg_launch_ms": round(avg_ms, 4),
                         "algorithmic_bytes_per_launch": int(avg_bytes),
                         "launches_per_step": round(dom[0] / args.steps, 2)},
            "propagation_ms_per_step": round(t_prop, 3),
            "per_launch_kind": {
                f"{KIND_NAMES[k[0]]}{'+inmask' if k[1] else ''}{'+rowmask' if k[2] else ''}":
                {"launches_per_step": round(v[0] / args.steps, 2), "avg_ms": round(v[1] / v[0], 4)}
                for k, v in sorted(per_kind.items())},
            "prune": bool(args.prune),
            "frontier_F1_rows": f1_rows,
            "recall": recall,
            "cpu_baseline": cpu,
            "setup_s": round(t_setup, 2),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
