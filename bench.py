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

Launch:
    python bench.py [--gpus N --steps K --warmup W]
With N > 1 and no WORLD_SIZE in the environment the script starts the N
ranks itself (torch.distributed.run as a child process; this parent never
touches the GPU) and exits with the ranks' status — the reference's
mp.spawn(demo, nprocs=world_size) entry (ddp_lgcn.py:760-768).  The
explicit form works too:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
--rehearse runs every rank on cuda:0 with gloo collectives (the N-rank code
path on a one-GPU box; not a throughput measurement).

Quality leg (--quality-steps S, default 3000): a second C2-sized graph with
community structure (kind='cluster'), S training steps of the same engine
from random init — with N > 1 through dist.DataParallel, every rank drawing B
triples from its user shard — then rank 0 computes Recall@20 / NDCG@20 with
trainer.py / metric.py semantics (the rank-0 evaluation of ddp_lgcn.py:
678-743) — reported beside the throughput, which is measured on the
structureless uniform graph where any recall is chance.

Parity leg (--parity 1): at N = 1 one more GPU step against the CPU oracle
from the same state; at N > 1 one more data-parallel step whose replicas must
be bitwise equal (digests all-gathered) and whose table must match, at 1e-4,
ONE single-process step of the union batch replayed on rank 0 from a snapshot
(dp_union_parity).  A failed check fails the run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import subprocess
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
PMC_FILE = os.path.join("profiles", "pmc_prop_kernel.json")
# MI355X_MICROARCH.md: the achievable HBM stream rate of a read/write kernel
# (the "HBM-honest" reference for counter bytes; the spec peak is above)
HBM_STREAM_GBS = 6290.0
PARITY_TOL = 1e-4  # north_star: output embeddings within 1e-4 rel fp32 of the CPU path
# C5 (d = 256, 11.26 GB tables: no Infinity-Cache help): the latest committed
# full-size bench line, read at run time (no_cache_reference)
C5_NO_CACHE_FILE = os.path.join("profiles", "round6_final_bench_c5_1gpu.json")


def parse(argv=None):
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
    ap.add_argument("--cpu-k", type=int, default=3, help="timed CPU steps after 1 warm-up")
    ap.add_argument("--quality-steps", type=int, default=3000,
                    help="training steps of the Recall@20 leg (every rank, B triples each; "
                         "with N > 1 through dist.DataParallel, rank 0 evaluates); 0: off")
    ap.add_argument("--quality-clusters", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=2020)
    ap.add_argument("--prune", type=int, default=1,
                    help="frontier pruning (1) or every layer on every row (0)")
    ap.add_argument("--dp-mode", default="auto", choices=["auto", "sparse", "dense", "sharded"],
                    help="gradient exchange (dist.DataParallel); auto = sparse and sharded "
                         "both timed during the warm-up on this job's ranks, the faster kept")
    ap.add_argument("--calib-steps", type=int, default=3,
                    help="timed warm-up steps per exchange mode for --dp-mode auto")
    ap.add_argument("--shard-chunks", type=int, default=4,
                    help="row blocks of the sharded last layer (all-gather overlap)")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP timing events (propagation launches, collectives) on every "
                         "k-th timed step only: each event record leaves the GPU idle ~5 us, "
                         "so events on every step would add ~1 %% to the timed step")
    ap.add_argument("--parity", type=int, default=1,
                    help="N=1: one more GPU step checked against the CPU oracle from the "
                         "same table / Adam state / triples; N>1: one more data-parallel "
                         "step checked bitwise across the replicas and, on rank 0, against "
                         "one single-process step on the union batch (the run fails above "
                         "1e-4)")
    ap.add_argument("--rehearse", action="store_true",
                    help="all ranks on cuda:0, gloo collectives (N-rank path on one GPU)")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.steps < 1:
        ap.error("--steps must be >= 1")
    return args


# ---------------------------------------------------------------- launcher

def launch_command(n: int, argv: list[str]) -> list[str]:
    """The child command that starts n ranks of this script (one process
    per GPU) with the same arguments.  The rendezvous store binds its own
    port (c10d endpoint 127.0.0.1:0): no port is picked here and handed
    over, so no other process can take it in between."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0",
            "--local-addr=127.0.0.1", os.path.abspath(__file__), *argv]


def needs_launch(args, env=os.environ) -> bool:
    return args.gpus > 1 and "WORLD_SIZE" not in env


def launch(args, argv: list[str], runner=subprocess.run) -> int:
    """Start the ranks as a child process tree and return their exit status.
    Nothing here initialises HIP: the parent only waits."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, host_threads() // args.gpus)))
    r = runner(launch_command(args.gpus, argv), env=env)
    return int(r.returncode)


def launch_selftest(args) -> None:
    """CPU-only rank body used by the launcher test: gloo rendezvous, one
    all-reduce, rank 0 prints one JSON line."""
    from furusato_recommend_amd.dist import init_distributed
    init_distributed("gloo", timeout_s=60)
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "sum": float(t)}), flush=True)
    dist.destroy_process_group()


# ---------------------------------------------------------------- host info

def host_threads() -> int:
    """CPU threads this process may actually use: the affinity mask, capped
    by a cgroup CPU quota (on the GPU box os.cpu_count() reports the whole
    host while the job's share is smaller)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, int(n))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def layer_bytes(n_nodes: int, nnz: int, d: int) -> int:
    """BASELINE.md §3 per-layer algorithmic bytes of the CPU propagation."""
    return nnz * d * 4 + nnz * 4 + (n_nodes + 1) * 4 + n_nodes * 4 + n_nodes * d * 4


def progress(msg: str) -> None:
    """A progress line on stderr (long legs keep a watchdog informed; the one
    JSON line stays alone on stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    """max|a - b| / max|b| over the whole tensor (the north_star's 1e-4
    relative fp32 bar; the same measure as tests/test_gpu_parity.py)."""
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def parity_snapshot(model, eng, emb, args, step_index: int, rank: int, world: int):
    """One more training step of the benchmarked engine, with everything the
    CPU oracle needs to take the SAME step copied to the host first: the
    table and the Adam moments / step count as they stand after the timed
    steps, the full layer-mean output of that table (all N rows), and the
    step's (u, p, n).  Then the GPU step itself: its loss and the table it
    leaves.  The oracle side runs in ``cpu_baseline``."""
    from furusato_recommend_amd.engine import sample_triples
    dev = emb.device
    B = args.batch
    u = torch.empty(B, dtype=torch.int32, device=dev)
    p, n = torch.empty_like(u), torch.empty_like(u)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    sample_triples(model.graph, B, args.seed, step_index * B, u, p, n, err, rank, world)
    ad = model.optim
    snap = {"emb0": emb.detach().cpu().clone(), "exp_avg": ad.exp_avg.cpu().clone(),
            "exp_avg_sq": ad.exp_avg_sq.cpu().clone(), "n_steps": int(ad.n_steps),
            "lr": ad.lr, "betas": ad.betas, "eps": ad.eps}
    out = eng.forward(emb)  # full layer mean of every row (unpruned)
    snap["out_gpu"] = out.cpu().clone()
    loss = eng.train_step(emb, model.optim, u, p, n, 1e-4)
    torch.cuda.synchronize()
    if int(err.item()) != 0:
        raise RuntimeError("sampler retry budget exhausted")
    snap.update(loss_gpu=float(loss.item()), emb1_gpu=emb.detach().cpu().clone(),
                users=u.cpu().numpy(), pos=p.cpu().numpy(), neg=n.cpu().numpy(),
                step_index=step_index)
    return snap


def oracle_parity(o, snap) -> dict:
    """The oracle takes the snapshot's step (model/lgcn.py:78-133 restated):
    same table, same Adam moments and step count, same triples.  Returns the
    relative errors of the full output, the stepped table and the loss."""
    with torch.no_grad():
        o.emb.copy_(snap["emb0"])
    o.optim.state[o.emb] = {"step": torch.tensor(float(snap["n_steps"])),
                            "exp_avg": snap["exp_avg"].clone(),
                            "exp_avg_sq": snap["exp_avg_sq"].clone()}
    grp = o.optim.param_groups[0]
    grp["lr"], grp["betas"], grp["eps"] = snap["lr"], tuple(snap["betas"]), snap["eps"]
    progress("parity: oracle full forward")
    out_cpu = o.propagated()
    progress("parity: oracle training step")
    loss_cpu = o.stageOne(snap["users"], snap["pos"], snap["neg"])
    r = {"rel_out": rel_err(snap["out_gpu"], out_cpu),
         "rel_emb_step": rel_err(snap["emb1_gpu"], o.emb.detach()),
         "rel_loss": abs(snap["loss_gpu"] - loss_cpu) / max(abs(loss_cpu), 1e-30),
         "loss_gpu": snap["loss_gpu"], "loss_cpu": loss_cpu,
         "rows": int(snap["emb0"].shape[0]), "tol": PARITY_TOL,
         "what": f"GPU training step {snap['step_index']} (after the timed steps) vs the CPU "
                 "oracle from the same table, Adam moments and step count on the same "
                 "(u, p, n): rel = max|gpu - cpu| / max|cpu| over every row of the "
                 "layer-mean output (before the step) and of the table after it"}
    r["ok"] = bool(max(r["rel_out"], r["rel_emb_step"], r["rel_loss"]) < PARITY_TOL)
    return r


# ------------------------------------------------- data-parallel parity leg

def _coll(t: torch.Tensor, backend: str, dev) -> torch.Tensor:
    """A tensor in the place the backend's collectives take it (RCCL: the
    device ``dev``; gloo: the host)."""
    return t.to(dev) if backend == "nccl" else t.cpu()


def replica_digest(*ts: torch.Tensor) -> torch.Tensor:
    """16-byte BLAKE2b digest of the tensors' bytes (uint8 [16], host): two
    replicas are bitwise equal iff their digests are (up to hash collision)."""
    import hashlib
    h = hashlib.blake2b(digest_size=16)
    for t in ts:
        h.update(t.detach().contiguous().cpu().view(torch.uint8).numpy().data)
    return torch.frombuffer(bytearray(h.digest()), dtype=torch.uint8)


def dp_union_parity(dp, emb: torch.Tensor, adam, users, pos, neg, decay: float, replay,
                    tol: float = PARITY_TOL) -> dict:
    """Proof that the N-rank step is the single-process step of the union
    batch (the reference's intent: ddp_lgcn.py:669-673 steps every rank's
    own batch through one shared model).  Collective: every rank calls it.

    Every rank snapshots the table and the Adam state (in ``sharded`` mode
    the moments are gathered first: each rank's are current on its own rows
    only), then takes one ``dp.step`` on its own (u, p, n).  Afterwards
      * every rank hashes its table and (gathered) Adam moments; the digests
        are all-gathered and must be identical — the replicas are bitwise
        one model;
      * rank 0 gathers every rank's triples, and ``replay(snap, U, P, N) ->
        (table, loss)`` takes ONE single-process step from the snapshot on
        the concatenated union batch (rank-major order); its table must be
        within ``tol`` (rel, max-abs) of the data-parallel table and its loss
        of the mean of the ranks' losses.
    Returns the record on rank 0 (``ok`` = all of it), a short one on the
    others."""
    world, rank = dp.world, dp.rank
    backend = dist.get_backend(dp.group)
    dev = emb.device
    dp.gather_optimizer_state()  # (no-op unless sharded moments are stale)
    snap = {"emb0": emb.detach().clone(), "exp_avg": adam.exp_avg.detach().clone(),
            "exp_avg_sq": adam.exp_avg_sq.detach().clone(), "n_steps": int(adam.n_steps)}
    trip = torch.stack([torch.as_tensor(x).to(torch.int32).reshape(-1)
                        for x in (users, pos, neg)])  # [3, B]
    allt = _coll(torch.empty(world * 3, trip.shape[1], dtype=torch.int32), backend, dev)
    dist.all_gather_into_tensor(allt, _coll(trip, backend, dev), group=dp.group)
    allt = allt.view(world, 3, -1)
    loss = dp.step(users, pos, neg, decay)
    dp.gather_optimizer_state()
    lsum = _coll(torch.as_tensor(loss, dtype=torch.float32).detach().reshape(1).clone(),
                 backend, dev)
    dist.all_reduce(lsum, group=dp.group)
    dig = torch.cat([replica_digest(emb), replica_digest(adam.exp_avg, adam.exp_avg_sq)])
    digs = _coll(torch.empty(world * dig.numel(), dtype=torch.uint8), backend, dev)
    dist.all_gather_into_tensor(digs, _coll(dig, backend, dev), group=dp.group)
    digs = digs.cpu().view(world, -1)
    tab_equal = bool((digs[:, :16] == digs[0, :16]).all())
    mom_equal = bool((digs[:, 16:] == digs[0, 16:]).all())
    r = {"world_size": world, "backend": backend, "mode": dp.mode,
         "replicas_bitwise_equal": tab_equal, "moments_bitwise_equal": mom_equal,
         "table_digest": digs[0, :16].numpy().tobytes().hex()}
    if rank != 0:
        return r
    allt = allt.cpu()
    U, P, N = (allt[:, k, :].reshape(-1) for k in range(3))
    emb1, loss1 = replay(snap, U, P, N)
    loss_dp = float(lsum.cpu()[0]) / world
    r.update(rel_emb_step=rel_err(emb, emb1),
             rel_loss=abs(loss_dp - float(loss1)) / max(abs(float(loss1)), 1e-30),
             loss_dp=loss_dp, loss_union=float(loss1), union_batch=int(U.numel()),
             rows=int(emb.shape[0]), tol=tol,
             what=f"one {world}-rank data-parallel step ({dp.mode} exchange) vs ONE "
                  f"single-process step on the union batch of all ranks' triples from the same "
                  "table / Adam state (rank 0): rel = max|dp - union| / max|union| over the whole "
                  "table; replicas' tables and Adam moments compared bitwise by digest")
    r["ok"] = bool(tab_equal and mom_equal and r["rel_emb_step"] < tol and r["rel_loss"] < tol)
    return r


def engine_replay(graph, args, world: int, decay: float, adam_like):
    """``replay`` for dp_union_parity on the GPU: a fresh PropagationEngine
    sized for the union batch (world x B triples) takes one train_step from
    the snapshot's table and Adam state."""
    from furusato_recommend_amd.engine import AdamState, PropagationEngine

    def replay(snap, U, P, N):
        dev = graph.device
        eng = PropagationEngine(graph, args.dim, args.layers, world * args.batch,
                                prune=bool(args.prune))
        e = snap["emb0"].to(dev).clone()
        ad = AdamState(e, adam_like.lr, adam_like.betas, adam_like.eps)
        ad.exp_avg.copy_(snap["exp_avg"])
        ad.exp_avg_sq.copy_(snap["exp_avg_sq"])
        ad.n_steps = snap["n_steps"]
        loss = eng.train_step(e, ad, U.to(dev), P.to(dev), N.to(dev), decay)
        torch.cuda.synchronize()
        return e, float(loss.item())
    return replay


def cpu_baseline(ds, args, users, pos, neg, snap=None):
    """The CPU oracle (torch fp32) on a bounded sample of the same workload,
    timed per BASELINE.md §3: one warm-up training step, then the mean of K
    full training steps (B triples each, full C2 graph); the 3-layer forward
    the same way (warmed by the warm-up step).  With ``snap`` (parity_snapshot)
    the oracle starts from the GPU's table and Adam state and its warm-up step
    is the parity step: the same step the GPU took, compared element-wise."""
    from oracle.lightgcn_oracle import OracleLightGCN, forward
    threads = host_threads()
    torch.set_num_threads(threads)
    o = OracleLightGCN(ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, args.dim,
                       args.layers, 1e-3, 1e-4, seed=args.seed,
                       emb=None if snap is None else snap["emb0"])
    K = max(1, args.cpu_k)
    res = {"cores": threads, "threads": threads, "os_cpu_count": os.cpu_count(),
           "kind": "port", "cpu": cpu_model(), "warmup": 1, "k": K}
    parity = None
    if snap is not None:
        parity = oracle_parity(o, snap)  # the warm-up step
        users, pos, neg = snap["users"], snap["pos"], snap["neg"]
    if args.cpu_baseline == "step":
        if parity is None:
            progress("cpu baseline: warm-up step")
            o.stageOne(users, pos, neg)  # warm-up
        ts = []
        for i in range(K):
            t0 = time.perf_counter()
            o.stageOne(users, pos, neg)
            ts.append(time.perf_counter() - t0)
            progress(f"cpu baseline: step {i + 1}/{K} {ts[-1]:.1f} s")
        t_step = sum(ts) / K
        res.update(value=round(len(users) / t_step, 3), unit="positive-edges/s",
                   step_s=round(t_step, 3), step_s_each=[round(t, 3) for t in ts],
                   sample=f"1 warm-up + mean of {K} full training steps (B={len(users)}) of "
                          f"the C2 workload (3-layer fwd+bwd+Adam over "
                          f"{ds.n_users + ds.m_items} nodes, {2 * ds.trainDataSize} "
                          f"adjacency entries)")
    else:
        with torch.no_grad():
            forward(o.emb, o.ei, ds.n_users, args.layers, o.div)  # warm-up
    tf = []
    with torch.no_grad():
        for i in range(K):
            t0 = time.perf_counter()
            forward(o.emb, o.ei, ds.n_users, args.layers, o.div)
            tf.append(time.perf_counter() - t0)
            progress(f"cpu baseline: forward {i + 1}/{K} {tf[-1]:.1f} s")
    t_fwd = sum(tf) / K
    nbytes = args.layers * layer_bytes(ds.n_users + ds.m_items, 2 * ds.trainDataSize, args.dim)
    res.update(forward_s=round(t_fwd, 3),
               forward_gbs=round(nbytes / t_fwd / 1e9, 3))
    if args.cpu_baseline == "forward":
        res.update(value=round(1.0 / t_fwd, 4), unit="forward passes/s",
                   sample=f"1 warm-up + mean of {K} 3-layer full-graph forwards of the C2 graph")
    return res, parity


def pmc_traffic(args):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    passes (rocprofv3 FETCH_SIZE / WRITE_SIZE, gfx950 correction; the
    counters cannot be read from inside this process)."""
    path = os.path.join(ROOT, PMC_FILE)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        j = json.load(f)
    kname = f"prop_kernel<{args.dim}, {({32: 2, 64: 4, 128: 4, 256: 8}).get(args.dim, 1)}, 0, false, false>"
    if (c2_workload(args) and j.get("workload") == f"C2-{args.kind}-d{args.dim}-L{args.layers}"
            and kname in j.get("kernel", "")):
        return j.get("hbm_bytes_per_launch"), f"{PMC_FILE} ({j.get('round', j.get('tag', 'r05'))})"
    return None, None


def hbm_counter(traffic, avg_ms):
    """The HBM-honest figure beside the algorithmic roofline: the PMC
    counter bytes of the dominant launch over its live duration, against the
    spec peak and the achievable stream rate.  At C2 the 25.6 MB item table
    and part of the user rows are served from Infinity Cache / L2, so the
    algorithmic rate (roofline.frac) can reach the spec peak while the
    counter rate stays near the stream rate."""
    if not traffic or not avg_ms:
        return None
    rate = traffic / (avg_ms * 1e-3) / 1e9
    return {"counter_GBps": round(rate, 1), "frac_of_peak": round(rate / HBM_PEAK_GBS, 4),
            "stream_GBps": HBM_STREAM_GBS, "frac_of_stream": round(rate / HBM_STREAM_GBS, 4),
            "no_cache_reference_c5": no_cache_reference()}


def no_cache_reference(path: str = C5_NO_CACHE_FILE) -> dict | None:
    """The HBM-honest roofline: C5's full launch (d = 256, 11.26 GB per
    table, far beyond Infinity Cache) from the committed C5 bench line."""
    try:
        with open(os.path.join(ROOT, path)) as f:
            j = next(json.loads(ln) for ln in f if ln.lstrip().startswith("{"))
        r = j["roofline"]
    except (OSError, StopIteration, KeyError, ValueError):
        return None
    return {"achieved_GBps": r["achieved"], "frac_of_peak": r["frac"],
            "avg_launch_ms": r["avg_launch_ms"],
            "algorithmic_bytes_per_launch": r["algorithmic_bytes_per_launch"], "source": path}


def c2_workload(args) -> bool:
    return (args.users, args.items, args.edges) == (1_000_000, 100_000, 20_000_000)


# ---------------------------------------------------------------- quality leg

def train_then_evaluate(step, steps: int, evaluate_fn, rank: int, world: int, sync=None,
                        group=None):
    """The quality leg's loop, rank-symmetric: ``steps`` calls of
    ``step(i)`` on every rank (a data-parallel step when world > 1), then
    rank 0 alone evaluates (``evaluate_fn()``) while the others wait at a
    barrier — the reference's DDP loop with its rank-0 evaluation
    (ddp_lgcn.py:669-743).  Returns (evaluation or None, train seconds)."""
    sync = sync or (lambda: None)
    sync()
    t = time.perf_counter()
    for i in range(steps):
        step(i)
        if (i + 1) % 500 == 0:
            sync()
            if rank == 0:
                progress(f"quality leg: {i + 1}/{steps} training steps")
    sync()
    t = time.perf_counter() - t
    res = None
    if rank == 0:
        progress("quality leg: evaluating Recall@20")
        res = evaluate_fn()
    if world > 1:
        dist.barrier(group=group)
    return res, t


def quality_leg(args, dev, steps: int, rank: int = 0, world: int = 1, dp_mode: str = "sparse"):
    """Recall@20 that measures something: train the same engine on a
    C2-sized graph with community structure (items i % K == user u % K with
    probability 0.9), `steps` steps of B triples per rank from the on-device
    sampler (each rank from its user shard; with world > 1 through
    dist.DataParallel in the exchange mode the throughput leg settled on),
    then rank 0 runs the evaluation path (trainer.py:115-187 semantics).
    Collective when world > 1; returns the record on rank 0, None elsewhere."""
    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.dist import DataParallel
    from furusato_recommend_amd.engine import sample_triples
    from furusato_recommend_amd.evaluate import evaluate
    t0 = time.perf_counter()
    if rank == 0:
        progress("quality leg: building the community graph")
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=7, kind="cluster",
                            n_clusters=args.quality_clusters, p_in=0.9, test_frac=0.1)
    if rank == 0:
        progress("quality leg: graph built")
    torch.manual_seed(args.seed)
    cfg = {"recdim": args.dim, "layer": args.layers, "lr": 1e-3, "decay": 1e-4,
           "device": str(dev), "bpr_batch_size": args.batch, "prune": bool(args.prune)}
    model = LightGCN(cfg, ds)
    eng, emb = model.engine, model.all_embedding.weight.data
    dp = DataParallel(eng, emb, model.optim, mode=dp_mode,
                      chunks=args.shard_chunks) if world > 1 else None
    B = args.batch
    u = torch.empty(B, dtype=torch.int32, device=dev)
    p, n = torch.empty_like(u), torch.empty_like(u)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    r0 = evaluate(model, ds.testDict, topks=(20,)) if rank == 0 else None

    def step(i):
        sample_triples(model.graph, B, args.seed + 1, i * B, u, p, n, err, rank, world)
        if dp is None:
            eng.train_step(emb, model.optim, u, p, n, cfg["decay"])
        else:
            dp.step(u, p, n, cfg["decay"])
    r, t_train = train_then_evaluate(step, steps,
                                     lambda: evaluate(model, ds.testDict, topks=(10, 20)),
                                     rank, world, sync=torch.cuda.synchronize)
    if int(err.item()) != 0:
        raise RuntimeError("sampler retry budget exhausted")
    if rank != 0:
        return None
    mean_deg = ds.trainDataSize / ds.n_users
    return {"recall@20": float(r["recall"][1]), "ndcg@20": float(r["ndcg"][1]),
            "recall@10": float(r["recall"][0]), "recall@20_at_init": float(r0["recall"][0]),
            "chance_recall@20": round(20.0 / (ds.m_items - mean_deg), 7),
            "test_users": len(ds.testDict), "train_steps": steps, "batch_per_rank": B,
            "global_batch": B * world, "ranks": world,
            "trained_by": (f"dist.DataParallel ({dp.mode} exchange), {world} ranks, "
                           "rank 0 evaluates" if dp is not None else "one engine"),
            "lr": 1e-3, "train_s": round(t_train, 2), "leg_s": round(time.perf_counter() - t0, 2),
            "graph": f"cluster: {args.users} x {args.items} / {args.edges} edges, "
                     f"{args.quality_clusters} communities, p_in 0.9, seed 7"}


# ---------------------------------------------------------------- main

def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if needs_launch(args):
        sys.exit(launch(args, argv))
    if args.launch_selftest:
        return launch_selftest(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    gpu = 0 if args.rehearse else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        from furusato_recommend_amd.dist import init_distributed
        init_distributed("gloo" if args.rehearse else "nccl", dev)
        world = dist.get_world_size()

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
    dp = DataParallel(eng, emb, model.optim, mode=args.dp_mode,
                      chunks=args.shard_chunks) if world > 1 else None
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
    calib = None
    if dp is not None and args.dp_mode == "auto":
        # both exchanges timed on this job's own ranks and links (extra
        # warm-up steps: ordinary training steps, untimed for the metric)
        nxt = [args.warmup]

        def run_step():
            step(nxt[0])
            nxt[0] += 1
        calib = dp.calibrate(run_step, steps=args.calib_steps)
        progress(f"dp calibration: {calib}")
    t_base = args.warmup if calib is None else nxt[0]
    dp_mode = dp.mode if dp is not None else "none"
    ag_ms = dp.time_table_allgather() if (dp is not None and calib is None
                                          and dp.mode == "sharded") else None
    torch.cuda.synchronize()
    # the live launch timing: HIP events on the launch stream around every
    # propagation launch (and collective) of every k-th timed step — an event
    # record idles the GPU for ~5 us (round-6 trace: ~50 us per C2 step with
    # events on all 12 records), so the other steps run without them
    every = max(1, args.event_every)
    prop_ev, comm_ev = [], []
    sampled = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j, i in enumerate(range(t_base, t_base + args.steps)):
        on = j % every == every - 1 or (args.steps < every and j == args.steps - 1)
        sampled += int(on)
        eng.prop_events = prop_ev if on else None
        if dp is not None:
            dp.comm_events = comm_ev if on else None
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    events, eng.prop_events = prop_ev, None
    comm = None
    if dp is not None:
        from furusato_recommend_amd.dist import _elapsed_ms
        comm_ms = dp._max_over_ranks(_elapsed_ms(comm_ev) / sampled)
        dp.comm_events = None
        xb = dp.exchange_bytes_per_rank(B)
        table = emb.numel() * emb.element_size()
        if calib is not None:
            ag_ms = calib["table_allgather_ms"]
        comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                "mode": dp_mode, "comm_ms_per_step": round(comm_ms, 4),
                "comm_note": "exposed exchange time on the compute stream (HIP events), max "
                             "over ranks: the blocking seed all-gather / all-reduce, plus in "
                             "sharded mode the table all-gather left after the overlapped "
                             "last layer",
                "exchange_bytes_per_rank": int(xb),
                "exchange_bytes_note": "bytes each rank receives per step",
                "algbw_GBps": (round(xb / (comm_ms * 1e-3) / 1e9, 2) if comm_ms > 0 else None),
                "table_allgather_ms": ag_ms,
                "table_allgather_algbw_GBps": (round(table / (ag_ms * 1e-3) / 1e9, 2)
                                               if ag_ms else None),
                "shard_chunks": args.shard_chunks if dp_mode == "sharded" else None,
                "calibration": calib}
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64,
                         device="cpu" if args.rehearse else dev)
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
    t_prop = sum(v[1] for v in per_kind.values()) / sampled
    dom = per_kind.get((0, False, False), [1, 1.0, 0])
    avg_ms = dom[1] / dom[0]
    avg_bytes = dom[2] / dom[0]
    achieved = avg_bytes / (avg_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args)

    snap = None
    dp_parity = None
    if rank == 0 and world == 1 and args.parity:
        progress("parity: GPU step from a host snapshot of the table and Adam state")
        snap = parity_snapshot(model, eng, emb, args, t_base + args.steps, rank, world)
    elif world > 1 and args.parity:
        if rank == 0:
            progress("parity: one data-parallel step vs the union batch replayed on rank 0")
        i = t_base + args.steps
        sample_triples(model.graph, B, args.seed, i * B, u, p, n, err, rank, world)
        dp_parity = dp_union_parity(dp, emb, model.optim, u, p, n, cfg["decay"],
                                    engine_replay(model.graph, args, world, cfg["decay"],
                                                  model.optim))
        if rank == 0:
            progress(f"parity: {dp_parity}")

    qsteps = max(0, args.quality_steps)
    recall = None
    if qsteps > 0:
        del model, eng, emb, dp
        torch.cuda.empty_cache()
        recall = quality_leg(args, dev, qsteps, rank, world, dp_mode)

    cpu = parity = None
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        cpu, parity = cpu_baseline(ds, args, u.cpu().numpy(), p.cpu().numpy(),
                                   n.cpu().numpy(), snap)
    elif snap is not None:
        from oracle.lightgcn_oracle import OracleLightGCN
        torch.set_num_threads(host_threads())
        o = OracleLightGCN(ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, args.dim,
                           args.layers, 1e-3, 1e-4, emb=snap["emb0"])
        parity = oracle_parity(o, snap)
    if dp_parity is not None:
        parity = dp_parity

    if rank == 0:
        value = world * args.steps * B / dt
        c2 = (args.users, args.items, args.edges, args.dim, args.layers) == \
            (1_000_000, 100_000, 20_000_000, 64, 3)
        wl = ("C2" if c2 else "custom") + (
            f": LightGCN {args.layers}-layer d={args.dim}, synthetic {args.users} users x "
            f"{args.items} items / {args.edges} edges ({args.kind})")
        par = (f"dp{world} rehearsal: {world} ranks on one GPU, gloo collectives"
               if args.rehearse else
               f"dp{world} (user-sharded, RCCL {dp_mode} gradient exchange)")
        line = {
            "metric": f"BPR positive-edges/sec (LightGCN-{args.layers} d={args.dim}, "
                      f"{args.users} x {args.items} / {args.edges} edges)",
            "value": round(value, 1),
            "unit": "positive-edges/s",
            "n_gpus": 1 if args.rehearse else world,
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
                       "ranks": world, "parallelism": par},
            "roofline": {"bound": "hbm",
                         "kernel": DOMINANT.replace("D, UNROLL", f"{args.dim}, "
                                                    f"{ {32: 2, 64: 4, 128: 4, 256: 8}.get(args.dim, 1)}"),
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "avg_launch_ms": round(avg_ms, 4),
                         "algorithmic_bytes_per_launch": int(avg_bytes),
                         "launches_per_step": round(dom[0] / sampled, 2),
                         "timed_steps_sampled": sampled},
            "roofline_hbm_counter": hbm_counter(traffic, avg_ms),
            "propagation_ms_per_step": round(t_prop, 3),
            "per_launch_kind": {
                f"{KIND_NAMES[k[0]]}{'+inmask' if k[1] else ''}{'+rowmask' if k[2] else ''}":
                {"launches_per_step": round(v[0] / sampled, 2), "avg_ms": round(v[1] / v[0], 4)}
                for k, v in sorted(per_kind.items())},
            "prune": bool(args.prune),
            "frontier_F1_rows": f1_rows,
            "recall": recall,
            "parity": parity,
            "cpu_baseline": cpu,
            "setup_s": round(t_setup, 2),
        }
        if comm is not None:
            line["comm"] = comm
        if args.rehearse:
            line["rehearsal"] = True
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and not parity.get("ok", True):
        raise SystemExit(f"parity above {PARITY_TOL}: {parity}")


if __name__ == "__main__":
    main()
