"""Data-parallel training driver: replaces ``demo`` of ddp_lgcn.py:625-746
(LightGCN) and ddp_sage.py:754-878 (GraphSAGE); SASRec runs through it too.

The reference's loop, per rank (one process per GPU, ``mp.spawn``):

  * load ``checkpoints/ddp_<model>_<suffix>.pth`` at start (:660);
  * per epoch, ``UniformSample`` (:541-582: TRAIN_ITERATIVE x trainDataSize
    candidate users, a positive each, kept while that positive was kept
    fewer than POSITIVE_NUM_LIMIT times, a rejection-sampled negative), a
    barrier, then ``OneEpoch`` over minibatches (:668-676);
  * every TEST_SPAN epochs, on rank 0: save the checkpoint and evaluate
    Recall / Precision / NDCG / HR / Coverage @10, @20 over TEST_COUNT
    batches of test users (:678-743).

What differs here, and why:

  * Each rank samples on device from ITS OWN user shard (u ≡ rank mod W;
    ``engine.sample_epoch_capped`` for models with a CSR ``graph``, uniform
    shard users + ``sample_pairs`` for SASRec) with an independent counter
    stream, and the epoch's TRAIN_ITERATIVE x trainDataSize candidates are
    split over the ranks (``epoch_split``, default): the union of the ranks'
    batches is one epoch of the single-process sampler.  (The reference's
    ranks each draw a full epoch from their own numpy seed, 1000 x rank.)
  * Every step goes through the gradient exchange of ``dist.DataParallel``
    (LightGCN) or ``dist.DenseGradDataParallel`` (GraphSAGE, SASRec), so the
    replicas train on the union batch.  The reference's ranks never
    exchanged gradients (``ddp_model.module.OneEpoch``, :673 — DDP's hooks
    are bypassed), i.e. they trained W independent models.
  * The ranks must take the same number of steps with equal batch sizes
    (every step is a collective): after sampling, the kept-triple counts are
    reduced with MIN and every rank keeps that many (the capped sampler keeps
    a data-dependent number per rank).
  * Before a checkpoint every rank takes part in ``gather_optimizer_state``
    (the sharded exchanges keep Adam moments — and under ``fetch`` the table
    rows — current on the owner only), then rank 0 saves and evaluates while
    the others wait at a barrier.  The checkpoint file holds the model's
    ``state_dict`` exactly as the reference's (its ``.pth`` files load and
    vice versa); the optimizer state and the epoch go to ``<path>.train``.
  * Collectives run under the process group's finite timeout
    (``dist.init_distributed``), not the reference's unbounded barriers.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

# ddp_lgcn.py:34-37 / ddp_sage.py:34-37
POSITIVE_NUM_LIMIT = 3000
TRAIN_ITERATIVE = 3
TEST_COUNT = 100
TEST_SPAN = 5


def _rank_world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _reduce_int(x: int, op, group=None, device=None) -> int:
    """One int reduced over the ranks (MIN / MAX / SUM); gloo reduces on the
    host, RCCL on the device."""
    if not (dist.is_available() and dist.is_initialized()):
        return int(x)
    dev = device if (device is not None and dist.get_backend(group) == "nccl") else "cpu"
    t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=op, group=group)
    return int(t.item())


def _reduce_float(x: float, group=None, device=None) -> float:
    """Mean of a float over the ranks."""
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    dev = device if (device is not None and dist.get_backend(group) == "nccl") else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item()) / dist.get_world_size(group)


def optimizer_states(model) -> list:
    """The model's optimizer state objects (each with state_dict /
    load_state_dict): LightGCN / MF ``optim``, GraphSAGE / SASRec ``optims``."""
    if getattr(model, "optims", None) is not None:
        return list(model.optims)
    if getattr(model, "optim", None) is not None:
        return [model.optim]
    return []


def wrap(model, group=None, mode: str | None = None, **kw):
    """The data-parallel wrapper for ``model``: ``DataParallel`` over the
    fused engine (LightGCN; ``mode`` = its gradient exchange) or
    ``DenseGradDataParallel`` for the autograd models (``mode`` = the id
    table's exchange)."""
    from .dist import DataParallel, DenseGradDataParallel, HostDataParallel
    if hasattr(model, "engine") and hasattr(model, "all_embedding"):
        return DataParallel(model.engine, model.all_embedding.weight.data, model.optim,
                            group=group, mode=mode or "auto", **kw)
    if hasattr(model, "host_grad") and getattr(model, "on_host", False):
        return HostDataParallel(model, group=group)  # MF on the host (C1)
    if hasattr(model, "engine") and hasattr(model, "_table"):
        # MF on the GPU: the fused engine with no propagation layers
        return DataParallel(model.engine, model._table, model.optim, group=group,
                            mode=mode or "sparse", **kw)
    return DenseGradDataParallel(model, group=group, table_exchange=mode, **kw)


def coverage(top: np.ndarray, m_items: int, k: int) -> float:
    """metric.py:142-147: distinct items among every user's top-k / m_items."""
    if top.size == 0:
        return 0.0
    return float(np.unique(top[:, :k]).size) / float(m_items)


class DPTrainer:
    """The ddp_lgcn.py / ddp_sage.py epoch driver on the data-parallel
    wrappers (module docstring).  ``sampler(epoch) -> (users, pos, neg)``
    and ``evaluator(model) -> (metrics, top_items)`` default to the model's
    on-device sampler and ``evaluate.evaluate``; tests pass their own."""

    def __init__(self, config: dict, dataset, model, dp=None, group=None, sampler=None,
                 evaluator=None, log=None):
        self.config = config
        self.dataset = dataset
        self.model = model
        self.group = group
        self.rank, self.world = _rank_world(group)
        self.dp = dp if dp is not None else wrap(model, group, config.get("dp_mode"))
        self.batch = int(config.get("bpr_batch_size", 2048))
        self.decay = float(config.get("decay", 1e-4))
        self.seed = int(config.get("seed", 2020))
        self.test_span = int(config.get("test_span", TEST_SPAN))
        self.train_iterative = int(config.get("train_iterative", TRAIN_ITERATIVE))
        self.cap = int(config.get("positive_num_limit", POSITIVE_NUM_LIMIT))
        self.epoch_split = bool(config.get("epoch_split", True))
        self.topks = tuple(config.get("topks", (10, 20)))
        self.test_batch = int(config.get("test_u_batch_size", 1000))
        self.test_count = config.get("test_count", TEST_COUNT)
        self.checkpoint_path = config.get("checkpoint_path")
        self.sampler = sampler or self._default_sampler
        self.evaluator = evaluator or self._default_evaluator
        self.log = log or (lambda rec: None)
        self.device = getattr(model, "device", None)
        self.epoch = 0
        self.history = []
        self.max_recall = 0.0

    # ------------------------------------------------------------ sampling
    def _n_candidates(self) -> int:
        n = self.train_iterative * int(self.dataset.trainDataSize)
        return -(-n // self.world) if self.epoch_split else n

    def _default_sampler(self, epoch: int):
        """This rank's triples of one epoch, on device."""
        m = self.model
        nc = self._n_candidates()
        if getattr(m, "graph", None) is not None and hasattr(m.graph, "csr_ptr"):
            from .engine import sample_epoch_capped
            return sample_epoch_capped(m.graph, nc, self.cap, seed=self.seed,
                                       offset=epoch * nc, shard=self.rank, n_shards=self.world)
        if hasattr(m, "sample_pairs"):  # SASRec: shard users, device (pos, neg)
            g = torch.Generator().manual_seed(self.seed * 1_000_003 + epoch * 7919 + self.rank)
            n_shard = -(-(int(m.n_user) - self.rank) // self.world)
            n = self.train_iterative * int(self.dataset.trainDataSize) // self.world \
                if self.epoch_split else self.train_iterative * int(self.dataset.trainDataSize)
            users = torch.randint(0, max(n_shard, 1), (n,), generator=g) * self.world + self.rank
            pn = m.sample_pairs(users.to(m.device), seed=self.seed, offset=epoch * n * self.world
                                + self.rank * n)
            return users, pn[0], pn[1]
        raise TypeError(f"no default sampler for {type(m).__name__}: pass sampler=")

    def equalise(self, users, pos, neg):
        """Every rank keeps the same number of triples (the MIN over ranks),
        so the ranks take the same steps with equal batch sizes."""
        k = _reduce_int(len(users), dist.ReduceOp.MIN, self.group, self.device)
        return users[:k], pos[:k], neg[:k]

    # ------------------------------------------------------------- training
    def _accumulates(self) -> bool:
        """DataParallel (the fused engine) sums the loss on the device and
        HostDataParallel on the host; the autograd wrappers return each
        step's loss."""
        return bool(getattr(self.dp, "accumulates_loss", hasattr(self.dp, "engine")))

    def _step(self, u, p, n, acc):
        if self._accumulates():
            return self.dp.step(u, p, n, self.decay, acc)
        return self.dp.step(u, p, n)

    def train_one_epoch(self, epoch: int) -> dict:
        """ddp_lgcn.py:669-676: sample, barrier, OneEpoch (the mean loss over
        len // B + 1 as model/lgcn.py:135-151)."""
        t0 = time.perf_counter()
        users, pos, neg = self.equalise(*self.sampler(epoch))
        if self.world > 1:
            dist.barrier(group=self.group)
        n = len(users)
        B = self.batch
        acc = torch.zeros(1, dtype=torch.float32,
                          device=self.device if self.device is not None else "cpu")
        total = 0.0
        for i in range(0, n, B):
            loss = self._step(users[i:i + B], pos[i:i + B], neg[i:i + B], acc)
            if not self._accumulates():
                total += float(loss)
        loss_rank = (float(acc[0]) if self._accumulates() else total) / (n // B + 1)
        rec = {"epoch": epoch, "triples_per_rank": n, "steps": -(-n // B) if n else 0,
               "loss": _reduce_float(loss_rank, self.group, self.device),
               "loss_rank": loss_rank, "epoch_s": round(time.perf_counter() - t0, 3)}
        return rec

    # ---------------------------------------------------------- checkpoints
    def _train_state_path(self):
        return self.checkpoint_path + ".train"

    def save_checkpoint(self, epoch: int):
        """Rank 0, after gather_optimizer_state on every rank: the model's
        state_dict at ``checkpoint_path`` (the reference's .pth format,
        ddp_lgcn.py:681) and the optimizer states + epoch beside it."""
        path = self.checkpoint_path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        sd = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        torch.save(sd, path + ".tmp")
        os.replace(path + ".tmp", path)
        opt = [_to_cpu(s.state_dict()) for s in optimizer_states(self.model)]
        torch.save({"epoch": int(epoch), "optim": opt, "max_recall": float(self.max_recall),
                    "counters": _step_counters(self.model)},
                   self._train_state_path() + ".tmp")
        os.replace(self._train_state_path() + ".tmp", self._train_state_path())

    def load_checkpoint(self) -> bool:
        """ddp_lgcn.py:658-661 on every rank: the model state (and, when
        present, the optimizer states and the next epoch).  Loaded with
        weights_only=True."""
        path = self.checkpoint_path
        if not path or not os.path.exists(path):
            return False
        sd = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(sd)
        tp = self._train_state_path()
        if os.path.exists(tp):
            st = torch.load(tp, map_location="cpu", weights_only=True)
            for s, o in zip(optimizer_states(self.model), st["optim"]):
                s.load_state_dict(o)
            self.epoch = int(st["epoch"]) + 1
            self.max_recall = float(st.get("max_recall", 0.0))
            for k, v in st.get("counters", {}).items():
                setattr(self.model, k, int(v))
        _after_load(self.model, self.dp)
        return True

    # ----------------------------------------------------------- evaluation
    def _default_evaluator(self, model):
        from .evaluate import evaluate
        td = self.dataset.testDict
        if self.test_count is not None:  # ddp_lgcn.py:710: TEST_COUNT batches
            keep = sorted(td)[: int(self.test_count) * self.test_batch]
            td = {u: td[u] for u in keep}
        return evaluate(model, td, self.topks, self.test_batch, return_topk=True)

    def test(self, epoch: int):
        """Collective: every rank gathers its sharded state, rank 0 saves the
        checkpoint and evaluates, the others wait (ddp_lgcn.py:678-743)."""
        gather = getattr(self.dp, "gather_optimizer_state", None)
        if gather is not None:
            gather()
        res = None
        if self.rank == 0:
            if self.checkpoint_path:
                self.save_checkpoint(epoch)
            if hasattr(self.model, "eval"):
                self.model.eval()
            metrics, top = self.evaluator(self.model)
            if hasattr(self.model, "train"):
                self.model.train()
            res = {k: np.asarray(v, dtype=np.float64).tolist() for k, v in metrics.items()}
            res["coverage"] = [coverage(np.asarray(top), int(self.dataset.m_items), k)
                               for k in self.topks]
            if res["recall"][0] > self.max_recall:
                self.max_recall = res["recall"][0]
        if self.world > 1:
            dist.barrier(group=self.group)
        return res

    def fit(self, epochs: int) -> list:
        """Resume from the checkpoint if one exists, then ``epochs`` epochs
        with a checkpoint + evaluation every ``test_span`` (epoch % span ==
        0, as ddp_lgcn.py:678)."""
        self.load_checkpoint()
        end = self.epoch + int(epochs)
        while self.epoch < end:
            i = self.epoch
            rec = self.train_one_epoch(i)
            if i % self.test_span == 0:
                rec["metrics"] = self.test(i)
            self.history.append(rec)
            self.log(rec)
            self.epoch += 1
        return self.history


def _to_cpu(x):
    if torch.is_tensor(x):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x


# Per-step counters that seed a model's step (GraphSAGE: every step's tree
# and dropout seed is _step_seed * 7919 + _calls): kept in the .train file
# so a resumed run draws what an uninterrupted one would have.
STEP_COUNTERS = ("_calls", "_step_seed")


def _step_counters(model) -> dict:
    return {k: int(getattr(model, k)) for k in STEP_COUNTERS
            if isinstance(getattr(model, k, None), int)}


def _after_load(model, dp):
    """After a checkpoint load: a fused engine forgets its cached dinv ⊙ E;
    the wrappers' row-sharded state is whole again on every rank, and so is
    a ``fetch``-exchange table (the loaded table is the full one)."""
    if getattr(model, "table_stale", False):
        model.table_stale = False
    eng = getattr(model, "engine", None)
    if eng is not None and hasattr(eng, "invalidate_prescaled"):
        eng.invalidate_prescaled()
    for s in optimizer_states(model):
        if hasattr(s, "stale_rows"):
            s.stale_rows = False
    if dp is not None and hasattr(dp, "_norms_next"):
        dp._norms_next = None


# ------------------------------------------------------------------ launcher
# ``python -m furusato_recommend_amd.train_dp --model lgn --gpus 8 ...``
# replaces ``if __name__ == '__main__': mp.spawn(demo, nprocs=world_size)``
# (ddp_lgcn.py:760-768, ddp_sage.py:892-899).  With --gpus N > 1 and no
# WORLD_SIZE in the environment the parent starts torch.distributed.run as
# a child process (N ranks, one per GPU, 127.0.0.1 rendezvous) and exits
# with its status; the parent never touches the GPU.  Each rank builds the
# dataset and the model, wraps it and runs DPTrainer.fit.  Option names are
# the reference's (parse.py:4-64; ddp_lgcn.py:636-656 for the DDP values).

def parse_args(argv=None):
    import argparse
    ap = argparse.ArgumentParser(
        prog="python -m furusato_recommend_amd.train_dp",
        description="Data-parallel BPR training (ddp_lgcn.py / ddp_sage.py on MI355X)")
    ap.add_argument("--model", default="lgn", help="registry name: lgn | sage | sasrec | mf")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU)")
    ap.add_argument("--epochs", type=int, default=200, help="ddp_lgcn.py:667 range(200)")
    ap.add_argument("--bpr_batch", type=int, default=20000, help="per-rank batch (ddp_lgcn.py:646)")
    ap.add_argument("--recdim", type=int, default=32, help="ddp_lgcn.py:647")
    ap.add_argument("--layer", type=int, default=2, help="ddp_lgcn.py:648")
    ap.add_argument("--lr", type=float, default=1e-3, help="ddp_lgcn.py:653")
    ap.add_argument("--decay", type=float, default=1e-4, help="ddp_lgcn.py:645")
    ap.add_argument("--num_neighbors", type=int, default=5, help="GraphSAGE fanout per hop")
    ap.add_argument("--fanouts", default=None,
                    help="GraphSAGE fanout per hop as a list, e.g. [25,10] (C3)")
    ap.add_argument("--testbatch", type=int, default=1000, help="test_u_batch_size")
    ap.add_argument("--topks", default="[10,20]")
    ap.add_argument("--test_span", type=int, default=TEST_SPAN)
    ap.add_argument("--test_count", type=int, default=TEST_COUNT,
                    help="test batches per evaluation (ddp_lgcn.py:710); -1 = all users")
    ap.add_argument("--train_iterative", type=int, default=TRAIN_ITERATIVE)
    ap.add_argument("--positive_num_limit", type=int, default=POSITIVE_NUM_LIMIT)
    ap.add_argument("--seed", type=int, default=2020)
    ap.add_argument("--path", default="./checkpoints",
                    help="checkpoint directory: <path>/ddp_<model>_<suffix>.pth")
    ap.add_argument("--suffix", default="all")
    ap.add_argument("--data", default=None,
                    help="directory holding <suffix>/train<suffix>.txt and test<suffix>.txt "
                         "(dataloader.py format)")
    ap.add_argument("--synthetic", default=None,
                    help="n_users,m_items,n_edges[,kind] instead of --data "
                         "(SyntheticBipartite; kind uniform | zipf | cluster)")
    ap.add_argument("--dp_mode", default=None,
                    help="gradient exchange (LightGCN: auto | sparse | dense | sharded; "
                         "GraphSAGE / SASRec: the table exchange)")
    ap.add_argument("--backend", default=None, choices=("nccl", "gloo"),
                    help="default nccl (RCCL) on GPUs, gloo with --device cpu")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"))
    ap.add_argument("--rehearse", action="store_true",
                    help="every rank on cuda:0 over gloo (the N-rank path on one GPU)")
    ap.add_argument("--factory", default=None,
                    help="module:callable(config, dataset, rank, world) -> model, or a dict "
                         "with 'model' and optionally 'dp', 'sampler', 'evaluator' "
                         "(a model plugin outside the registry)")
    ap.add_argument("--log", default=None, help="rank 0 appends one JSON line per epoch here")
    return ap.parse_args(argv)


def needs_launch(args, env=os.environ) -> bool:
    return args.gpus > 1 and "WORLD_SIZE" not in env


def launch_command(args, argv: list) -> list:
    """torch.distributed.run with a c10d rendezvous whose store binds its own
    port (endpoint 127.0.0.1:0): no free port is picked here and handed over
    (another process could take it in between)."""
    import sys
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={args.gpus}", "--rdzv-backend=c10d",
            "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1",
            "-m", "furusato_recommend_amd.train_dp", *argv]


def launch(args, argv: list, runner=None) -> int:
    """Start the ranks as a child process tree (nothing here initialises
    HIP) and return their exit status."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join(p for p in (root, env.get("PYTHONPATH")) if p)
    if "OMP_NUM_THREADS" not in env:
        env["OMP_NUM_THREADS"] = str(max(1, min(os.cpu_count() or 1, 64) // args.gpus))
    r = (runner or subprocess.run)(launch_command(args, argv), env=env)
    return int(r.returncode)


def build_config(args, device: str) -> dict:
    import ast
    return {
        "device": device, "bpr_batch_size": args.bpr_batch, "recdim": args.recdim,
        "latent_dim_rec": args.recdim, "layer": args.layer, "lr": args.lr,
        "decay": args.decay, "num_neighbors": args.num_neighbors,
        "test_u_batch_size": args.testbatch, "topks": tuple(ast.literal_eval(args.topks)),
        "test_span": args.test_span,
        "test_count": None if args.test_count < 0 else args.test_count,
        "train_iterative": args.train_iterative,
        "positive_num_limit": args.positive_num_limit, "seed": args.seed,
        "suffix": args.suffix, "dp_mode": args.dp_mode,
        "checkpoint_path": os.path.join(args.path, f"ddp_{args.model}_{args.suffix}.pth"),
        **({"fanouts": list(ast.literal_eval(args.fanouts))} if args.fanouts else {}),
    }


def build_dataset(args, config: dict):
    from .dataloader import Loader, SyntheticBipartite
    if (args.data is None) == (args.synthetic is None):
        raise SystemExit("train_dp: give exactly one of --data DIR or --synthetic n,m,e[,kind]")
    if args.data is not None:
        return Loader({"suffix": args.suffix}, path=args.data)
    f = args.synthetic.split(",")
    kind = f[3] if len(f) > 3 else "uniform"
    return SyntheticBipartite(int(f[0]), int(f[1]), int(f[2]), seed=0, kind=kind)


def _resolve(spec: str):
    import importlib
    mod, _, fn = spec.partition(":")
    return getattr(importlib.import_module(mod), fn)


def run_rank(args) -> list:
    """One rank: process group (when launched with WORLD_SIZE), dataset,
    model, DPTrainer.fit; rank 0 prints one JSON line per epoch."""
    import json
    from .dist import init_distributed
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_cpu = args.device == "cpu"
    backend = args.backend or ("gloo" if (on_cpu or args.rehearse) else "nccl")
    if on_cpu:
        device = "cpu"
    else:
        device = f"cuda:{0 if args.rehearse else local}"
        torch.cuda.set_device(torch.device(device))
    if world > 1:
        init_distributed(backend, device=None if (on_cpu or backend == "gloo")
                         else torch.device(device))
    rank, _ = _rank_world()
    try:
        config = build_config(args, device)
        ds = build_dataset(args, config)
        torch.manual_seed(args.seed)
        parts = {}
        if args.factory:
            made = _resolve(args.factory)(config, ds, rank, world)
            parts = made if isinstance(made, dict) else {"model": made}
        else:
            from .register import MODELS
            if args.model not in MODELS:
                raise SystemExit(f"train_dp: unknown model {args.model!r} "
                                 f"(known: {sorted(MODELS)})")
            parts = {"model": MODELS[args.model](config, ds)}

        def log(rec):
            if rank != 0:
                return
            line = json.dumps({"model": args.model, "world": world, **rec})
            print(line, flush=True)
            if args.log:
                with open(args.log, "a") as f:
                    f.write(line + "\n")
        tr = DPTrainer(config, ds, parts["model"], dp=parts.get("dp"), sampler=parts.get("sampler"),
                       evaluator=parts.get("evaluator"), log=log)
        return tr.fit(args.epochs)
    finally:
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def main(argv=None) -> int:
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if needs_launch(args):
        return launch(args, argv)
    run_rank(args)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
