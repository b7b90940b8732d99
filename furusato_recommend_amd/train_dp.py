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
    from .dist import DataParallel, DenseGradDataParallel
    if hasattr(model, "engine") and hasattr(model, "all_embedding"):
        return DataParallel(model.engine, model.all_embedding.weight.data, model.optim,
                            group=group, mode=mode or "auto", **kw)
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
        """DataParallel (the fused engine) sums the loss on the device; the
        autograd wrappers return each step's loss."""
        return hasattr(self.dp, "engine")

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
        torch.save({"epoch": int(epoch), "optim": opt, "max_recall": float(self.max_recall)},
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


def _after_load(model, dp):
    """After a checkpoint load: a fused engine forgets its cached dinv ⊙ E;
    the wrappers' row-sharded state is whole again on every rank."""
    eng = getattr(model, "engine", None)
    if eng is not None and hasattr(eng, "invalidate_prescaled"):
        eng.invalidate_prescaled()
    for s in optimizer_states(model):
        if hasattr(s, "stale_rows"):
            s.stale_rows = False
    if dp is not None and hasattr(dp, "_norms_next"):
        dp._norms_next = None
