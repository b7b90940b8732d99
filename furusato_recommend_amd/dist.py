"""User-sharded data parallelism over RCCL (replaces ddp_lgcn.py:625-768).

One process per GPU (launched by torch.distributed.run).  Every rank holds a
full replica of the embedding table, the CSR and the optimizer state (C2:
282 MB per [N, D] tensor).  Per step each rank

  1. draws its own B triples on device from the users of its shard
     (u % world_size == rank; mirec_bpr_sample), so the union batch covers
     every user with no sampling collective;
  2. runs the full-graph forward and the BPR loss on its own batch, with
     its gradient seeds scaled by 1/world_size;
  3. exchanges gradients over RCCL (xGMI) so that every rank holds exactly
     the gradient of the union batch of world_size * B triples (the
     reference's DDP never synchronises gradients because it calls
     `.module.OneEpoch`, ddp_lgcn.py:673 — this is what it meant to do);
  4. applies Adam; replicas stay bit-identical because every rank applies
     the same reduced gradient to the same parameters.

Gradient exchange modes:
  * ``sparse`` (default): the backward is linear in the gradient seeds
    (dL/d out, non-zero on <= 3B rows per rank, plus the reg rows), so the
    union batch's gradient is the backward of the SUM of all ranks' seeds.
    Ranks all-gather their packed seeds (3B x (4 + 8D) bytes: 3.2 MB at
    B=2048, D=64) and merge them in rank order (mirec_seed_merge), then run
    the backward with Adam fused — 8x 3.2 MB over xGMI instead of an all-reduce
    of the 282 MB dense gradient.
  * ``dense``: SUM all-reduce of the dense gradient dE, then the dense Adam
    kernel (the textbook DDP exchange; kept for comparison).
  * ``sharded``: the sparse exchange, but the last backward layer and its
    fused Adam run only on this rank's rows i ≡ rank (mod W) — interleaved,
    not a contiguous block, so every shard holds its share of short user rows
    and long item rows; the optimizer state of the other rows is not touched
    here (ZeRO-1 style) — then the updated table is all-gathered (N x D x 4
    bytes per step, 282 MB at C2; in row blocks, each block's all-gather
    overlapping the next block's launch) and the next forward re-derives
    dinv ⊙ E.  It trades the replicated full last layer + Adam (1.6 ms at C2
    on every rank) for the all-gather, which pays once xGMI moves the table
    faster than that.  (DenseGradDataParallel below shards
    its id tables in contiguous row blocks instead: a reduce-scatter's
    natural layout.)
  * ``auto`` (default): ``sparse`` until ``calibrate`` has timed both
    ``sparse`` and ``sharded`` on the job's own ranks and links, then the
    faster of the two.
All modes give the gradient of the union batch; replicas stay bit-identical.

The initial parameters are broadcast from rank 0 (the DDP ctor broadcast,
ddp_lgcn.py:663).  The engine is duck-typed (forward / bpr / backward /
adam_step), so the CPU tests drive this exact driver with gloo and an
oracle-backed engine.  The forward is frontier-pruned to the rank's own
batch; after the sparse exchange the backward is pruned to the union seeds.
"""
from __future__ import annotations

import ctypes
import datetime
import os
import time

import torch
import torch.distributed as dist

# Watchdog on rendezvous and collectives (the reference's ranks hang
# forever on a barrier when one dies, ddp_lgcn.py:671).
DEFAULT_TIMEOUT_S = float(os.environ.get("MIREC_DIST_TIMEOUT_S", "300"))


def init_distributed(backend: str = "nccl", device: torch.device | None = None,
                     timeout_s: float = DEFAULT_TIMEOUT_S, **kw) -> None:
    """`dist.init_process_group` with a finite timeout (replaces the
    unbounded NCCL setup of ddp_lgcn.py:748-755).  A rank that dies or stalls
    makes the others raise after `timeout_s` seconds instead of hanging the
    job; for RCCL the same bound applies to every collective (the process
    group's watchdog)."""
    if backend == "nccl" and device is not None:
        kw.setdefault("device_id", device)
    dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)


def _elapsed_ms(events) -> float:
    """Sum of (start, end) HIP-event intervals in ms (events recorded on the
    stream the collectives synchronise with)."""
    return sum(a.elapsed_time(b) for a, b in events)


class DataParallel:
    """See the module docstring.  ``mode="auto"`` runs ``sparse`` until
    ``calibrate`` has timed both ``sparse`` and ``sharded`` steps on this
    job's ranks and links and switched to the faster one (the decision and
    both timings are kept in ``self.calibration``).  ``chunks`` (``sharded``)
    splits the last backward layer into that many row blocks; the finished
    rows of each block are all-gathered (``async_op``) while the next block
    is computed (the exchange overlapped with the last SpMM)."""

    MODES = ("auto", "sparse", "dense", "sharded")

    def __init__(self, engine, emb: torch.Tensor, adam, group=None, mode: str = "auto",
                 chunks: int | None = None):
        if mode not in self.MODES:
            raise ValueError(mode)
        self.requested = mode
        self.mode = "sparse" if mode == "auto" else mode
        self.engine = engine
        self.emb = emb
        self.adam = adam
        self.group = group
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.n_chunks = max(1, int(os.environ.get("MIREC_SHARD_CHUNKS", "4")
                                   if chunks is None else chunks))
        self.grad = None
        self.calibration = None
        # HIP-event intervals of the exchange, per step, when a list (bench.py):
        # (start, end) pairs on the current stream around every collective's
        # exposed part (blocking calls: the whole collective; the overlapped
        # table all-gather: from the last chunk's launch to the last unpack)
        self.comm_events = None
        if self.world > 1:
            dist.broadcast(emb.data, src=0, group=group)
        # the row shards' static lists and the N x D staging buffer: built
        # now for "sharded", on first use for "auto" (and dropped again when
        # the calibration keeps "sparse": 282 MB at C2, ~11 GB at C5)
        self._chunks = None
        self.last_rows = None
        if mode == "sharded":
            self._init_shard()
        self._mark_sharded_state(False)

    def _ensure_shard(self):
        if self._chunks is None:
            self._init_shard()

    def _free_shard(self):
        self._chunks = None
        self.last_rows = None

    # ------------------------------------------------------------ row shards
    def _init_shard(self):
        """This rank's rows i ≡ r (mod W) — interleaved, so every shard gets
        its share of both the short user rows and the long item rows (a
        contiguous split would give rank 0 only users: 0.5 vs 1.3 ms of last
        layer at W = 2).  Slot s of rank r is row r + s·W (S = ceil(N / W)
        slots).  The slots are cut into ``n_chunks`` blocks [s0, s1): block c
        covers rows [s0·W, s1·W), has its own static row lists (the last
        backward layer's launch for that block) and its own [W, s1 - s0, D]
        staging buffer, the output of one all-gather."""
        N, D = self.emb.shape
        W, r = self.world, self.rank
        S = (N + W - 1) // W
        C = max(1, min(self.n_chunks, S))
        bounds = [(c * S) // C for c in range(C + 1)]
        words = (N + 15) // 16 * 4
        dev = self.emb.device
        # (allocated whenever a process group exists: at W = 1 the collectives
        # still run, so a one-GPU job exercises the RCCL calls of the path)
        stage = torch.empty(W * S * D, dtype=self.emb.dtype, device=dev) \
            if self.distributed else None
        self._chunks = []
        off = 0
        for c in range(C):
            s0, s1 = bounds[c], bounds[c + 1]
            bm = torch.zeros(words, dtype=torch.int32, device=dev)
            bm.view(torch.uint8)[r + s0 * W: min(s1 * W, N): W] = 1
            st = None
            if stage is not None:
                st = stage[off: off + W * (s1 - s0) * D].view(W, s1 - s0, D)
                off += W * (s1 - s0) * D
            self._chunks.append((s0, s1, self.engine.static_row_lists(bm), st))
        self._S = S
        self.last_rows = [ch[2] for ch in self._chunks]

    def _pack(self, c: int, t: torch.Tensor):
        s0, s1, _, st = self._chunks[c]
        N, D = t.shape
        r, W = self.rank, self.world
        if t.is_cuda:
            from . import _lib
            from ._lib import check, lib
            check(lib.mirec_shard_pack(t.data_ptr(), N, D, W, r, s0, s1 - s0, st[r].data_ptr(),
                                       _lib.stream_handle()), "shard_pack")
            return
        rows = t[r + s0 * W: min(s1 * W, N): W]  # (host tensors: the CPU driver tests)
        st[r, : rows.shape[0]].copy_(rows)

    def _gather_chunk(self, c: int, async_op: bool):
        _, _, _, st = self._chunks[c]
        W, D = self.world, st.shape[2]
        return dist.all_gather_into_tensor(st.view(-1, D), st[self.rank], group=self.group,
                                           async_op=async_op)

    def _unpack(self, c: int, t: torch.Tensor, x0s: torch.Tensor | None = None):
        """Block c's rows of the other ranks from the staging buffer into
        ``t`` (and, with ``x0s``, dinv ⊙ those rows into x0s: the next
        forward's pre-scaled input)."""
        s0, s1, _, st = self._chunks[c]
        N, D = t.shape
        W = self.world
        if t.is_cuda:
            from . import _lib
            from ._lib import check, lib
            check(lib.mirec_shard_unpack(st.data_ptr(), N, D, W, self.rank, s0, s1 - s0,
                                         _lib.ptr(None if x0s is None else self.engine.g.dinv),
                                         t.data_ptr(), _lib.ptr(x0s), _lib.stream_handle()),
                  "shard_unpack")
            return
        e = min(s1 * W, N)
        full = (e - s0 * W) // W  # slots holding all W ranks' rows
        if full:
            t[s0 * W: s0 * W + full * W].view(full, W, D).copy_(st[:, :full].transpose(0, 1))
        for w in range(e - s0 * W - full * W):  # the ragged last row block
            t[s0 * W + full * W + w].copy_(st[w, full])

    def _gather_rows(self, t: torch.Tensor):
        """Every rank's shard rows of ``t`` [N, D] to every rank (in place):
        per block, pack rows r, r+W, ... into this rank's staging slot, one
        all-gather, then scatter slot w's rows back to w, w+W, ..."""
        if not self.distributed:
            return
        self._ensure_shard()
        for c in range(len(self._chunks)):
            self._pack(c, t)
            self._gather_chunk(c, async_op=False)
            self._unpack(c, t)

    def _mark_sharded_state(self, stale: bool):
        """Flag the Adam state whose moments are current on this rank's rows
        only (a state_dict() then raises instead of saving stale moments)."""
        if self.adam is not None:
            self.adam.stale_rows = stale

    def gather_optimizer_state(self):
        """After ``sharded`` steps each rank's Adam moments are current on its
        own rows only; bring every row's moments to every rank (collective:
        call it on every rank, e.g. before a checkpoint of the optimizer
        state)."""
        if self.adam is not None and getattr(self.adam, "stale_rows", False):
            self._gather_rows(self.adam.exp_avg)
            self._gather_rows(self.adam.exp_avg_sq)
            self._mark_sharded_state(False)

    def shard(self):
        """(shard, n_shards) for the on-device sampler."""
        return self.rank, self.world

    # ------------------------------------------------------------ exchange
    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def _exchange(self, keys, rows_p, rows_e):
        """One all-gather of [key | seed_p | seed_e] records (the int32 key
        travels bit-cast in the first float column), split back by rank-major
        row order."""
        D = rows_p.shape[1]
        rec = torch.cat([keys.view(torch.float32).unsqueeze(1), rows_p, rows_e], dim=1)
        allrec = self._all_gather(rec)
        return (allrec[:, 0].contiguous().view(torch.int32), allrec[:, 1:1 + D].contiguous(),
                allrec[:, 1 + D:].contiguous())

    def _event(self):
        if self.comm_events is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _note(self, a, b):
        if a is not None:
            self.comm_events.append((a, b))

    def exchange_bytes_per_rank(self, batch: int, mode: str | None = None) -> int:
        """Bytes one rank receives per step in ``mode`` (default: the current
        one): the seed records of the other W-1 ranks (3B x (1 + 2D) floats
        each), plus in ``sharded`` the other ranks' table rows ((W-1)/W of
        N x D floats), in ``dense`` a ring all-reduce's 2(W-1)/W of the
        gradient."""
        mode = mode or self.mode
        N, D = self.emb.shape
        W = self.world
        table = N * D * self.emb.element_size()
        seeds = (W - 1) * 3 * batch * (1 + 2 * D) * 4
        if mode == "sparse":
            return seeds
        if mode == "sharded":
            return seeds + (W - 1) * table // W
        return 2 * (W - 1) * table // W

    def step(self, users, pos, neg, decay: float, loss_accum=None):
        eng = self.engine
        out = eng.forward_for_batch(self.emb, users, pos, neg)
        loss = eng.bpr(out, self.emb, users, pos, neg, decay, loss_accum,
                       grad_scale=1.0 / self.world)
        if self.mode in ("sparse", "sharded"):
            keys, rows_p, rows_e = eng.export_seeds()
            if self.distributed:
                a = self._event()
                keys, rows_p, rows_e = self._exchange(keys, rows_p, rows_e)
                self._note(a, self._event())
            eng.import_seeds(keys, rows_p, rows_e)
            if self.mode == "sparse":
                eng.backward(self.emb, adam=self.adam)
            else:
                self._ensure_shard()
                works = []
                overlap = self.distributed

                def on_chunk(c):
                    if overlap:
                        self._pack(c, self.emb)
                        works.append(self._gather_chunk(c, async_op=True))
                eng.backward(self.emb, adam=self.adam, last_rows=self.last_rows,
                             on_chunk=on_chunk)
                a = self._event()
                # the unpack also writes dinv ⊙ E for the other ranks' rows
                # (the fused Adam wrote this rank's): no prescale pass follows
                x0s = getattr(eng, "x0s", None) if self.emb.is_cuda else None
                for c, w in enumerate(works):
                    w.wait()
                    self._unpack(c, self.emb, x0s)
                self._note(a, self._event())
                if x0s is not None and overlap and getattr(eng, "reuse_prescaled", False):
                    eng.mark_prescaled(self.emb)
                else:
                    eng.invalidate_prescaled()
                self._mark_sharded_state(self.world > 1)
        else:
            if self.grad is None:
                self.grad = torch.empty_like(self.emb)
            eng.backward(self.emb, grad_out=self.grad)
            if self.distributed:
                a = self._event()
                dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.group)
                self._note(a, self._event())
            eng.adam_step(self.emb, self.grad, self.adam)
        return loss

    # ------------------------------------------------------------ auto mode
    def _max_over_ranks(self, x: float) -> float:
        if not self.distributed:
            return x
        dev = self.emb.device if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def time_table_allgather(self, reps: int = 3) -> float:
        """Best-of-``reps`` ms of the sharded mode's table all-gather alone
        (every block, blocking, no packing), max over ranks: the link rate
        the ``sharded`` mode pays (algbw = N·D·4 B / this)."""
        if not self.distributed:
            return 0.0
        self._ensure_shard()
        best = float("inf")
        for _ in range(reps):
            torch.cuda.synchronize()  # (a CUDA table: time_table_allgather is GPU-only)
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for c in range(len(self._chunks)):
                self._gather_chunk(c, async_op=False)
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        return self._max_over_ranks(best)

    def _measure(self, mode: str, run_step, steps: int) -> float:
        """Wall ms per step of ``steps`` steps (after a barrier), max over ranks."""
        torch.cuda.synchronize()
        dist.barrier(group=self.group)
        t0 = time.perf_counter()
        for _ in range(steps):
            run_step()
        torch.cuda.synchronize()
        return self._max_over_ranks(1e3 * (time.perf_counter() - t0) / steps)

    def calibrate(self, run_step, steps: int = 2, measure=None,
                  force: bool = False) -> dict | None:
        """``auto``: run ``steps`` timed training steps (after one untimed
        one) in ``sparse`` and in ``sharded`` mode — ``run_step()`` performs
        one ``self.step`` on a fresh batch — take the max over ranks of each
        mode's time per step, switch to the faster mode and record both, with
        the table all-gather alone, in ``self.calibration``.  Every mode
        computes the union batch's update, so the steps taken here are
        ordinary training steps.  A no-op (None) unless mode was "auto" and
        W > 1 (``force``: also at W = 1, tests).  ``measure(mode, run_step,
        steps) -> ms`` replaces the wall clock (tests)."""
        if self.requested != "auto" or not self.distributed or (self.world == 1 and not force):
            return None
        measure = measure or self._measure
        ms = {}
        for m in ("sparse", "sharded"):
            self.mode = m
            run_step()
            ms[m] = float(measure(m, run_step, steps))
        choice = min(ms, key=ms.get)
        self.mode = choice
        self.gather_optimizer_state()  # no-op unless leaving sharded moments behind
        ag = self.time_table_allgather() if self.emb.is_cuda else 0.0
        if choice != "sharded":
            self._free_shard()
        table = self.emb.numel() * self.emb.element_size()
        self.calibration = {"sparse_ms_per_step": round(ms["sparse"], 4),
                            "sharded_ms_per_step": round(ms["sharded"], 4),
                            "steps_per_mode": steps, "choice": choice,
                            "table_allgather_ms": round(ag, 4),
                            "table_allgather_algbw_GBps":
                                round(table / (ag * 1e-3) / 1e9, 2) if ag > 0 else None}
        return self.calibration


class HostDataParallel:
    """Data parallelism for a model trained on the host (MF with
    device="cpu", configuration C1, under train_dp --device cpu; the
    reference's DDP over gloo).  The model exposes the two halves of its
    fused host step: ``host_grad(u, p, n, grad_scale)`` (the dense gradient
    into ``host_grad_buffer``) and ``host_adam()``.  Every rank computes its
    own batch's gradient scaled by 1/world_size, the gradients are SUM
    all-reduced, and every rank applies the same Adam step: the union
    batch's update, replicas bit-identical.  The initial table is broadcast
    from rank 0."""

    accumulates_loss = True  # step() adds the loss into the caller's accumulator

    def __init__(self, model, group=None):
        self.model = model
        self.group = group
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.comm_events = None
        if self.world > 1:
            for p in model.parameters():
                dist.broadcast(p.data, src=0, group=group)

    def step(self, users, pos, neg, decay: float | None = None, loss_accum=None):
        m = self.model
        loss = m.host_grad(users, pos, neg, grad_scale=1.0 / self.world)
        if self.distributed and self.world > 1:
            dist.all_reduce(m.host_grad_buffer, op=dist.ReduceOp.SUM, group=self.group)
        m.host_adam()
        if loss_accum is not None:
            loss_accum += loss
        return loss

    def gather_optimizer_state(self):
        """Nothing is sharded: every rank holds the whole state."""


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None, group=None):
    """all_to_all_single; CUDA tensors under gloo (CPU tests, one-GPU
    rehearsals) travel through host copies."""
    if inp.is_cuda and dist.get_backend(group) != "nccl":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def distinct_rows(ids: torch.Tensor, n_rows: int, lo: int = 0, hi: int = 0,
                  have: torch.Tensor | None = None, sync: bool = True):
    """Ascending distinct ids of the int32 device tensor ``ids`` in [0,
    n_rows) outside [lo, hi) (mirec_distinct_rows: byte map, block counts,
    ordered writes — no sort); one host sync for the count.  ``have`` (bool
    / uint8 [n_rows]): ids marked there are skipped, and the ids returned are
    marked (mirec_distinct_rows_unseen).  ``sync=False``: no host sync —
    returns (the n_rows-long output buffer, the count int32 [1] on the
    device)."""
    from . import _lib
    from ._lib import check, lib
    ids = ids.to(torch.int32).contiguous()
    dev = ids.device
    nb = int(lib.mirec_distinct_rows_workspace(int(n_rows)))
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
    out = torch.empty(max(int(n_rows), 1), dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    if have is None:
        check(lib.mirec_distinct_rows(ids.data_ptr(), ids.numel(), int(n_rows), int(lo), int(hi),
                                      out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(),
                                      _lib.stream_handle()), "distinct_rows")
    else:
        if have.numel() < n_rows or have.element_size() != 1 or not have.is_contiguous():
            raise ValueError("have: a contiguous 1-byte map of n_rows entries")
        check(lib.mirec_distinct_rows_unseen(ids.data_ptr(), ids.numel(), int(n_rows), int(lo),
                                             int(hi), have.data_ptr(), out.data_ptr(),
                                             cnt.data_ptr(), ws.data_ptr(), ws.numel(),
                                             _lib.stream_handle()), "distinct_rows_unseen")
    if not sync:
        return out, cnt
    return out[: int(cnt.item())]


def route_pack(ids: torch.Tensor, count: torch.Tensor, n_rows: int, parts: int, cap: int,
               blocks: torch.Tensor, stride: int) -> None:
    """The ascending ids (``count`` int32 [1] of them valid, on the device)
    as one block per owner at blocks[q·stride:]: [count_q, owner q's ids, ...
    up to cap] — an all-to-all with equal splits moves them and the counts
    travel in-band (mirec_route_pack; no host sync)."""
    from . import _lib
    from ._lib import check, lib
    if blocks.dtype != torch.int32 or not blocks.is_contiguous() or \
            blocks.numel() < (parts - 1) * stride + cap + 1:
        raise ValueError("blocks: contiguous int32 holding parts blocks of stride words")
    check(lib.mirec_route_pack(ids.data_ptr(), count.data_ptr(), ids.numel(), int(n_rows),
                               int(parts), int(cap), int(stride), blocks.data_ptr(),
                               _lib.stream_handle()), "route_pack")


def gather_rows_routed(table: torch.Tensor, blocks: torch.Tensor, parts: int, cap: int,
                       stride: int, out: torch.Tensor) -> None:
    """The owner side of route_pack's blocks (received from every source):
    out[...] = table rows of their ids in source order, the counts read on
    the device (mirec_gather_rows_routed); ``out`` holds parts·cap rows."""
    from . import _lib
    from ._lib import check, lib
    d = table.shape[1]
    if out.shape[0] < parts * cap or out.shape[1] != d or not out.is_contiguous():
        raise ValueError("out: contiguous [parts * cap, d]")
    if blocks.numel() < (parts - 1) * stride + cap + 1:
        raise ValueError("blocks shorter than parts blocks of stride words")
    check(lib.mirec_gather_rows_routed(table.data_ptr(), table.shape[0], blocks.data_ptr(),
                                       int(parts), int(cap), int(stride), d, out.data_ptr(),
                                       _lib.stream_handle()), "gather_rows_routed")


def export_stamped(tg, parts: int, ws: torch.Tensor | None = None):
    """The rows the table gradient ``tg`` (graphsage.TableGrad) stamped in its
    last accumulate, ascending, and their rows of S — with NO host sync: all
    enqueued on the current stream (mirec_stamped_rows, then a gather that
    reads the count on the device).  Returns (rows int32 [cap], vals [cap,
    d], counts int32 [1 + parts] = total then per owner block, workspace);
    the first counts[0] entries of rows / vals are valid, cap = the
    accumulate's entry count (bounds the distinct rows).  After an accumulate
    in the packed form (``tg.rows_parts`` = parts) its output is returned as
    it is: no scan, no gather."""
    from . import _lib
    from ._lib import check, lib
    if getattr(tg, "export", None) is not None:
        rows, vals, counts = tg.export
        tg.export = None
        if counts.numel() != 1 + parts:
            raise ValueError("table gradient exported for another world size")
        return rows, vals, counts, ws
    N, d, dev = tg.n_rows, tg.dim, tg.acc.device
    nb = max(int(lib.mirec_distinct_rows_workspace(N)), 16)
    if ws is None or ws.numel() < nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    cap = max(min(N, int(tg.entries)), 1)
    rows = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(1 + parts, dtype=torch.int32, device=dev)
    s = _lib.stream_handle()
    check(lib.mirec_stamped_rows(tg.stamp.data_ptr(), N, int(tg.gen), int(parts), rows.data_ptr(),
                                 counts.data_ptr(), ws.data_ptr(), ws.numel(), s), "stamped_rows")
    vals = torch.empty(cap, d, dtype=tg.acc.dtype, device=dev)
    check(lib.mirec_gather_rows_counted(tg.acc.data_ptr(), rows.data_ptr(), counts.data_ptr(), cap,
                                        d, vals.data_ptr(), s), "gather_rows_counted")
    return rows, vals, counts, ws


def scatter_rows(dst: torch.Tensor, ids: torch.Tensor, src: torch.Tensor) -> None:
    """dst[ids[i]] = src[i] (ids distinct int32; mirec_scatter_rows): the
    install of fetched rows (replaces index_copy_, ~2x its rate)."""
    from . import _lib
    from ._lib import check, lib
    n, d = src.shape
    if n == 0:
        return
    ids = ids.to(torch.int32).contiguous()
    check(lib.mirec_scatter_rows(src.contiguous().data_ptr(), ids.data_ptr(), n, d,
                                 dst.data_ptr(), _lib.stream_handle()), "scatter_rows")


def gather_rows(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """table[ids] for int32 ids (mirec_gather_rows): the owner side's
    gather of requested rows (replaces index_select)."""
    from . import _lib
    from ._lib import check, lib
    ids = ids.to(torch.int32).contiguous()
    n, d = ids.numel(), table.shape[1]
    out = torch.empty(n, d, dtype=table.dtype, device=table.device)
    if n:
        check(lib.mirec_gather_rows(table.data_ptr(), ids.data_ptr(), n, d, out.data_ptr(),
                                    _lib.stream_handle()), "gather_rows")
    return out


OWNER_ADAM_MAX_SOURCES = 64  # mirec_owner_adam's limit; more: owner_sum passes + adam_table


def owner_sum(sources, lo: int, n_own: int, d: int, device, ws: torch.Tensor | None = None):
    """S of the own row block from (ids int32, rows [n, d]) source blocks
    added in list order (each block's ids distinct) — bitwise the sequence of
    index_add_ calls, in one pass (mirec_owner_sum).  Returns (S [n_own, d],
    workspace)."""
    from . import _lib
    from ._lib import check, lib
    out = torch.empty(n_own, d, dtype=torch.float32, device=device)
    arr = (_lib.RowBlock * max(len(sources), 1))()
    keep = []
    for a, (ids, rows) in zip(arr, sources):
        ids, rows = ids.to(torch.int32).contiguous(), rows.contiguous()
        keep.append((ids, rows))
        a.ids, a.rows, a.n = ids.data_ptr(), rows.data_ptr(), ids.numel()
    nb = max(int(lib.mirec_owner_sum_workspace(len(sources), n_own)), 16)
    if ws is None or ws.numel() < nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=device)
    check(lib.mirec_owner_sum(arr, len(sources), int(lo), int(n_own), int(d), ws.data_ptr(),
                              ws.numel(), out.data_ptr(), _lib.stream_handle()), "owner_sum")
    return out, ws


def owner_adam(sources, lo: int, n_own: int, d: int, param: torch.Tensor,
               exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, coef: torch.Tensor,
               n_user: int, hp, norms: torch.Tensor | None = None,
               ws: torch.Tensor | None = None):
    """owner_sum + the table Adam of the own block in one pass
    (mirec_owner_adam: S is never stored; bitwise the two-step result).
    ``param`` / ``exp_avg`` / ``exp_avg_sq``: flat views starting at row
    ``lo``; at most 64 sources.  Returns the workspace."""
    from . import _lib
    from ._lib import check, lib
    arr = (_lib.RowBlock * max(len(sources), 1))()
    keep = []
    for a, (ids, rows) in zip(arr, sources):
        ids, rows = ids.to(torch.int32).contiguous(), rows.contiguous()
        keep.append((ids, rows))
        a.ids, a.rows, a.n = ids.data_ptr(), rows.data_ptr(), ids.numel()
    nb = max(int(lib.mirec_owner_sum_workspace(len(sources), n_own)), 16)
    if ws is None or ws.numel() < nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=param.device)
    sumsq = None
    if norms is not None:
        sumsq = torch.empty(int(lib.mirec_adam_table_sumsq_floats(n_own, d)),
                            device=param.device)
    check(lib.mirec_owner_adam(arr, len(sources), int(lo), int(n_own), int(d), param.data_ptr(),
                               exp_avg.data_ptr(), exp_avg_sq.data_ptr(), coef.data_ptr(),
                               int(n_user), ctypes.byref(hp), _lib.ptr(sumsq), _lib.ptr(norms),
                               ws.data_ptr(), ws.numel(), _lib.stream_handle()), "owner_adam")
    return ws


def route_ids(ids: torch.Tensor, n_rows: int, group=None):
    """Send every row id to the rank owning it (contiguous blocks of
    n_rows/W rows; ``ids`` ascending int32).  Returns (received ids in
    source-rank order, per-source counts, per-owner counts sent)."""
    W = dist.get_world_size(group)
    per = n_rows // W
    owner = torch.div(ids.long(), per, rounding_mode="floor").clamp_(max=W - 1)
    send = torch.bincount(owner, minlength=W)
    recv = torch.empty_like(send)
    _a2a(recv, send, group=group)
    sc, rc = send.tolist(), recv.tolist()
    rid = torch.empty(int(sum(rc)), dtype=ids.dtype, device=ids.device)
    _a2a(rid, ids.contiguous(), rc, sc, group=group)
    return rid, rc, sc


def route_rows(rows: torch.Tensor, vals: torch.Tensor, n_rows: int, group=None):
    """Send every (row id, value row) to the rank owning the row — rank q
    owns the contiguous block [q·n_rows/W, (q+1)·n_rows/W) — with one small
    all-to-all of the counts and two uneven all-to-alls (ids, rows).
    ``rows``: ascending int32 [n] (so each owner's rows are one contiguous
    block), ``vals`` [n, d].  Returns (ids [m], vals [m, d], per-source
    counts): the received blocks in source-rank order, each ascending."""
    rid, rc, sc = route_ids(rows, n_rows, group)
    rv = torch.empty(rid.numel(), vals.shape[1], dtype=vals.dtype, device=vals.device)
    _a2a(rv, vals.contiguous(), rc, sc, group=group)
    return rid, rv, rc


class DenseGradDataParallel:
    """Data parallelism for models trained through autograd (GraphSAGE,
    SASRec; replaces ddp_sage.py:754-878, which like ddp_lgcn.py never
    synchronised gradients).  Every rank samples its own user shard; the loss
    is scaled by 1/world_size and the gradients are SUM-reduced over RCCL
    between backward and the (HIP) Adam step: the small ones as one flattened
    all-reduce bucket.  The id table (563 MB at C3) has three routes:

    * ``table_exchange="routed"`` (default for a model with a sorted table
      gradient, ``model._tg``, whose rows divide by W): its gradient is
      G = c ⊙ W + S with the norm term c ⊙ W dense but identical on every
      rank (W is replicated, c = W x this rank's coefficient) and the tree
      term S non-zero only on the rows this rank's batch touched (~0.5 M of
      1.1 M at C3).  Each rank sends its touched rows of S to their owners
      (contiguous row blocks; ``route_rows``), the owner sums the received
      blocks in source-rank order and runs the fused table Adam
      (G formed in the kernel, mirec_adam_table) on its N/W rows, then one
      in-place all-gather of the table.  The dense gradient is never
      materialised; per rank ≈ (W-1)/W · (touched rows x (4 + 4d) B) in plus
      (W-1)/W of the table — against 2 (W-1)/W of the table for the
      reduce-scatter + all-gather of the dense gradient.
    * ``shard_optimizer`` with a materialised gradient
      (``table_exchange="dense"``): reduce-scatter by contiguous row shard,
      dense Adam on this rank's N/W rows, in-place all-gather (ZeRO-1).
    * otherwise: an in-place all-reduce and the replicated Adam.

    * ``table_exchange="fetch"`` (default for GraphSAGE, whose step exposes
      its sampled tree before the forward): the routed exchange without the
      all-gather.  Only the owner keeps its row block current; before each
      forward a rank fetches the current values of the rows its tree reads
      (~0.5 M distinct rows of 1.1 M at C3) from their owners — one
      all-to-all of row ids, one of rows back — and the table's slice norms
      (the loss's parameter-norm term) come from the owners' Adam partials
      (an all-gather of 2 floats per rank, summed in rank order).  Per rank
      ≈ (W-1)/W x (touched rows + tree rows) x (4 + 4d) B in, about half of
      the routed exchange at C3.  The local table is then stale outside the
      own block and the tree's rows: ``gather_optimizer_state()`` (also
      ``sync_table()``) all-gathers it before inference or a checkpoint.

    In the sharded routes the other rows' Adam moments are not kept here:
    ``gather_optimizer_state()`` brings them together (AdamState.state_dict
    raises until then)."""

    BUCKET_MIN = 1 << 20  # elements: gradients this large are reduced in place

    def __init__(self, model, group=None, shard_optimizer: bool | None = None,
                 table_exchange: str | None = None, microbatches: int | None = None,
                 fetch_group=None):
        self.model = model
        # fetch exchange: the step as this many micro-batches whose row
        # fetches and routed gradient rows overlap the other micro-batches'
        # compute (_pipelined_step); 1 = one tree per step
        self.microbatches = max(1, int(os.environ.get("MIREC_DP_MICROBATCHES", "1")
                                       if microbatches is None else microbatches))
        self.group = group
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        states = list(getattr(model, "optims", None) or [])
        self._states = {id(st.param): st for st in states if hasattr(st, "exp_avg")}
        self.shard_optimizer = (self.world > 1 and bool(self._states)
                                if shard_optimizer is None else bool(shard_optimizer))
        tg = getattr(model, "_tg", None)
        tstate = getattr(model, "_table_state", None)
        routable = (tg is not None and tstate is not None and id(tstate.param) in self._states
                    and tg.n_rows % self.world == 0 and not tg.atomic)
        fetchable = routable and hasattr(model, "sample_tree")
        if table_exchange is None:
            table_exchange = ("fetch" if fetchable else "routed" if routable else "dense") \
                if self.world > 1 else "dense"
        if table_exchange not in ("fetch", "routed", "dense"):
            raise ValueError(table_exchange)
        if table_exchange != "dense" and not routable:
            raise ValueError("routed / fetch table exchange needs a sorted table gradient "
                             "(model._tg) whose rows divide by the world size")
        if table_exchange == "fetch" and not fetchable:
            raise ValueError("fetch table exchange needs a model with a sampled tree (GraphSAGE)")
        self.table_exchange = table_exchange
        if tg is not None:
            # dense: the sorted table gradient is materialised as .grad so it
            # can be reduced; routed / fetch: it stays in its sparse form
            # (world 1: left as the caller set it)
            if self.world > 1 or table_exchange != "dense":
                tg.dense = table_exchange == "dense"
            model._tg_routed = table_exchange != "dense"
        self._norms_next = None  # fetch: the table's slice norms after the last update
        self._sharded = set()  # ids of the parameters whose Adam runs sharded
        self._ones = None      # the routed Adam's all-stamped shard
        self.comm_events = None  # (start, end) HIP events per collective (bench)
        self.last_exchange_bytes = 0
        self._sr_ws = None        # pipelined fetch: export_stamped's workspace
        self._os_ws = None        # routed / fetch: owner_sum's position maps
        self._side_stream = None  # pipelined fetch: the routed rows' stream
        # fetch exchange: the row fetches on a communicator of their own, so
        # micro-batch 0's rows travel while the later micro-batches' id
        # exchanges (on `group`) run — one communicator would queue them
        # behind the fetch.  With the default group it is created here
        # (collectively: every rank constructs this object); with a caller's
        # subgroup the caller passes ``fetch_group`` (a second group over the
        # same ranks — dist.new_group must run on every process), else the
        # fetches share ``group`` (same results, no overlap).
        self._fetch_group = fetch_group
        self._counts_host = None  # pipelined fetch: the planner's pinned counts
        self._fetch_side = None  # pipelined fetch: the fetched rows' stream
        self._have = None  # pipelined fetch: rows fetched for an earlier micro-batch
        if (fetch_group is None and group is None and self.distributed and self.world > 1
                and table_exchange == "fetch"):
            self._fetch_group = dist.new_group()
        if self.world > 1:
            for p in model.parameters():
                dist.broadcast(p.data, src=0, group=group)

    def _event(self):
        if self.comm_events is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _note(self, a, b):
        if a is not None:
            self.comm_events.append((a, b))

    def _shardable(self, p) -> bool:
        g = p.grad
        return (self.shard_optimizer and id(p) in self._states and g.dim() >= 1
                and g.shape[0] % self.world == 0 and g.is_contiguous()
                and p.data.is_contiguous())

    @torch.no_grad()
    def _sharded_adam(self, p):
        """Reduce-scatter p.grad by row shard, Adam on this rank's rows, then
        all-gather p in place; p.grad is consumed (set to None)."""
        from . import _lib
        from ._lib import check, lib
        from .engine import _note_raw_write
        g = p.grad
        st = self._states[id(p)]
        n = g.numel() // self.world
        lo = self.rank * n
        a = self._event()
        if dist.get_backend(self.group) == "nccl":
            shard = torch.empty(n, dtype=g.dtype, device=g.device)
            dist.reduce_scatter_tensor(shard, g.view(-1), op=dist.ReduceOp.SUM, group=self.group)
        else:  # gloo (CPU tests, one-GPU rehearsal): all-reduce, keep this rank's rows
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            shard = g.view(-1)[lo:lo + n]
        self._note(a, self._event())
        hp = st.next_hparams()
        _note_raw_write()
        pf = p.data.view(-1)
        ea, es = st.exp_avg.view(-1), st.exp_avg_sq.view(-1)
        check(lib.mirec_adam_dense(pf[lo:].data_ptr(), shard.data_ptr(), ea[lo:].data_ptr(),
                                   es[lo:].data_ptr(), n, ctypes.byref(hp),
                                   _lib.stream_handle()), "adam_dense(shard)")
        a = self._event()
        dist.all_gather_into_tensor(pf, pf[lo:lo + n], group=self.group)
        self._note(a, self._event())
        self.last_exchange_bytes += 2 * (self.world - 1) * n * g.element_size()
        p.grad = None
        self._sharded.add(id(p))
        st.stale_rows = self.world > 1
        tg = getattr(self.model, "_tg", None)
        if tg is not None:
            tg.pending = False  # the step of the table gradient is done

    @torch.no_grad()
    def routed_export(self):
        """This rank's touched table rows (ascending int32) and their rows of
        S, the sparse term of the table gradient (a host sync: the count)."""
        tg = self.model._tg
        rows = torch.nonzero(tg.stamp == tg.gen).view(-1).to(torch.int32)
        return rows, tg.acc.index_select(0, rows.long())

    @torch.no_grad()
    def routed_adam(self, rid, rv, counts, norms: torch.Tensor | None = None):
        """Owner side of the routed exchange: S of the own row block from the
        received (ids, rows) blocks — added in source-rank order, each block's
        rows distinct, so no two adds meet one address in a launch — then the
        fused table Adam (G = W·c ⊙ table + S formed in the kernel) on the
        own rows only; with ``norms`` [2] the updated block's user / item slice
        norms are written there (the kernel's fixed-order partials)."""
        self._owner_adam([(rid, rv, counts)], self._union_coef(self.model._tg.coef), norms)

    def _union_coef(self, coef: torch.Tensor) -> torch.Tensor:
        """The union's norm coefficient: the SUM of the ranks' (each scales
        with its own 1/B, graphsage.py:333-336, so ranks with uneven batches —
        a short last batch — differ); 2 floats."""
        coef = coef.clone()
        if self.distributed:
            dist.all_reduce(coef, op=dist.ReduceOp.SUM, group=self.group)
        return coef

    @torch.no_grad()
    def _owner_adam(self, blocks, coef: torch.Tensor, norms: torch.Tensor | None = None):
        """S of the own row block from received (ids, rows, per-source
        counts) blocks, added in list order and source-rank order within a
        block (each source's rows distinct), then the fused table Adam with
        the union coefficient ``coef`` on the own rows."""
        from . import _lib
        from ._lib import check, lib
        from .engine import _note_raw_write
        tg, st = self.model._tg, self.model._table_state
        p = st.param
        N, d = p.shape
        n_own = N // self.world
        lo = self.rank * n_own
        sources = []
        for rid, rv, counts in blocks:
            off = 0
            for c in counts:
                if c:
                    sources.append((rid[off:off + c], rv[off:off + c]))
                off += c
        n_user = min(max(tg.n_user - lo, 0), n_own)
        hp = st.next_hparams()
        pf = p.data.view(-1)
        ea, es = st.exp_avg.view(-1), st.exp_avg_sq.view(-1)
        if len(sources) <= OWNER_ADAM_MAX_SOURCES:  # fused: S never stored
            self._os_ws = owner_adam(sources, lo, n_own, d, pf[lo * d:], ea[lo * d:],
                                     es[lo * d:], coef, n_user, hp, norms, self._os_ws)
            _note_raw_write()
            tg.pending = False
            self._sharded.add(id(p))
            st.stale_rows = self.world > 1
            return
        s_own, self._os_ws = owner_sum(sources, lo, n_own, d, p.device, self._os_ws)
        if self._ones is None or self._ones.numel() != n_own:
            self._ones = torch.ones(n_own, dtype=torch.int32, device=p.device)
        sumsq = None
        if norms is not None:
            sumsq = torch.empty(int(lib.mirec_adam_table_sumsq_floats(n_own, d)),
                                device=p.device)
        check(lib.mirec_adam_table(pf[lo * d:].data_ptr(), ea[lo * d:].data_ptr(),
                                   es[lo * d:].data_ptr(), coef.data_ptr(), n_user,
                                   s_own.data_ptr(), self._ones.data_ptr(), 1, n_own, d,
                                   ctypes.byref(hp), _lib.ptr(sumsq), _lib.ptr(norms),
                                   _lib.stream_handle()),
              "adam_table(shard)")
        _note_raw_write()
        tg.pending = False
        self._sharded.add(id(p))
        st.stale_rows = self.world > 1

    @torch.no_grad()
    def _routed_table_step(self):
        """The ``routed`` exchange + fused Adam of the id table (class doc)."""
        p = self.model._table_state.param
        N, d = p.shape
        W = self.world
        n_own = N // W
        lo = self.rank * n_own
        rows, vals = self.routed_export()
        a = self._event()
        # (the collectives run at W = 1 too: a one-GPU job exercises them)
        rid, rv, counts = route_rows(rows, vals, N, self.group)
        self._note(a, self._event())
        self.last_exchange_bytes += (sum(counts) - counts[self.rank]) * (4 + d * p.element_size())
        if self.table_exchange == "fetch":
            own = torch.empty(2, device=p.device)
            self.routed_adam(rid, rv, counts, norms=own)
            # the full table's slice norms: Σ over the owners' blocks of
            # norm², in rank order (identical on every rank)
            sq = own * own
            allp = torch.empty(W, 2, device=p.device)
            a = self._event()
            dist.all_gather_into_tensor(allp.view(-1), sq, group=self.group)
            self._note(a, self._event())
            tot = allp[0].clone()
            for q in range(1, W):
                tot += allp[q]
            self._norms_next = tot.sqrt()
            if self.distributed and W > 1:
                self.model.table_stale = True  # until sync_table()
            return
        self.routed_adam(rid, rv, counts)
        if self.distributed:
            pf = p.data.view(-1)
            a = self._event()
            dist.all_gather_into_tensor(pf, pf[lo * d:(lo + n_own) * d], group=self.group)
            self._note(a, self._event())
        self.last_exchange_bytes += (W - 1) * n_own * d * p.element_size()

    @torch.no_grad()
    def fetch_rows(self, tree):
        """``fetch``: before the forward, the current values of the rows the
        tree reads that lie outside this rank's block, from their owners (one
        all-to-all of ids, one of rows back), written into the local table;
        and the table's slice norms of the last update for the forward."""
        m = self.model
        if self._norms_next is not None:
            m._norm_cache = (self._norms_next, m._norm_token())
            self._norms_next = None
        if not self.distributed or self.world == 1:
            return
        p = m._table_state.param
        N, d = p.shape
        n_own = N // self.world
        lo = self.rank * n_own
        ids = torch.cat([g for g, _ in tree.groups])
        need = distinct_rows(ids, N, lo, lo + n_own)
        a = self._event()
        req, rc, sc = route_ids(need, N, self.group)
        rows = gather_rows(p.data, req)
        got = torch.empty(need.numel(), d, dtype=p.dtype, device=p.device)
        _a2a(got, rows, sc, rc, group=self.group)
        self._note(a, self._event())
        scatter_rows(p.data, need, got)
        self.last_exchange_bytes += need.numel() * d * p.element_size() + \
            (sum(rc) - rc[self.rank]) * 4

    # ---------------------------------------------- pipelined fetch exchange
    # The step as C micro-batches (GraphSAGE.stageOne(chunks=C)): every
    # micro-batch's tree is sampled first, so the ids of all C read sets are
    # routed to their owners at once and the owners gather all requested rows
    # from the current table up front (the table changes only in this step's
    # Adam); micro-batch k + 1's rows then travel (async all-to-all) while
    # micro-batch k computes, and micro-batch k's table-gradient rows leave
    # for their owners (async) while k + 1 computes.  The owner adds the
    # received blocks in (micro-batch, source rank) order and steps its row
    # block once.  Rows fetched for micro-batch k are not fetched again for
    # later ones (same table version).  Under gloo the transfers run
    # synchronously (same arithmetic, no overlap).

    def _a2a_async(self, out, inp, out_splits, in_splits, group=None):
        group = self.group if group is None else group
        if dist.get_backend(group) == "nccl":
            return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group,
                                          async_op=True)
        _a2a(out, inp, out_splits, in_splits, group=group)
        return None

    @torch.no_grad()
    def _plan_fetch(self, trees, st):
        """Route every micro-batch's read set with no host round trip in the
        planning: each read set (distinct rows outside the own block, rows
        of earlier micro-batches skipped) is packed into fixed-capacity
        blocks per owner with its count in-band (route_pack; capacity = the
        smaller of the tree's row count and the largest owner block, so no
        count can exceed it), an all-to-all with equal splits moves the
        blocks, the owners gather the requested rows reading the counts on
        the device (gather_rows_routed), and the send / receive counts go to
        pinned host memory behind an event.  The host reads micro-batch k's
        counts only when it issues k's rows (the uneven all-to-all needs its
        splits): micro-batch 0's at the end of the planning, while the
        device still plans the later micro-batches; the rows leave on a
        stream of their own that waits only for their gather
        (_fetch_issue)."""
        m = self.model
        if self._norms_next is not None:
            m._norm_cache = (self._norms_next, m._norm_token())
            self._norms_next = None
        st["fetch"] = []
        if not self.distributed or self.world == 1:
            return
        p = m._table_state.param
        N, d = p.shape
        W, C = self.world, len(trees)
        n_own = N // W
        lo = self.rank * n_own
        # the micro-batches' fetched-rows map: kept, cleared per step (a
        # 1-byte fill of the kept buffer: ~4 us against ~16 for torch.zeros)
        if self._have is None or self._have.numel() != N:
            self._have = torch.empty(N, dtype=torch.uint8, device=p.device)
        have = self._have
        have.zero_()
        a = self._event()
        if self._counts_host is None or len(self._counts_host) < C or \
                self._counts_host[0].shape != (2, W):
            self._counts_host = [torch.empty(2, W, dtype=torch.int32, pin_memory=p.is_cuda)
                                 for _ in range(max(C, 1))]
        for k, tree in enumerate(trees):
            ids = torch.cat([g for g, _ in tree.groups])
            cap = max(1, min(N - (W - 1) * n_own, ids.numel()))
            seg = 1 + cap
            buf, cnt = distinct_rows(ids, N, lo, lo + n_own, have=have if C > 1 else None,
                                     sync=False)
            send = torch.empty(W * seg, dtype=torch.int32, device=p.device)
            route_pack(buf, cnt, N, W, cap, send, seg)
            recv = torch.empty_like(send)
            _a2a(recv, send, group=self.group)  # equal splits: one block of cap + 1 words a peer
            host = self._counts_host[k]
            host.copy_(torch.stack((send.view(W, seg)[:, 0], recv.view(W, seg)[:, 0])),
                       non_blocking=True)
            counted = torch.cuda.Event() if p.is_cuda else None
            if counted is not None:
                counted.record()
            out = torch.empty(W * cap, d, dtype=p.dtype, device=p.device)
            gather_rows_routed(p.data, recv, W, cap, seg, out)  # owner side: the current rows
            gathered = torch.cuda.Event() if p.is_cuda else None
            if gathered is not None:
                gathered.record()
            st["fetch"].append({"buf": buf, "out": out, "cap": cap, "host": host,
                                "counted": counted, "gathered": gathered, "work": None})
            self.last_exchange_bytes += (W - 1) * seg * 4
        self._fetch_issue(0, st)
        self._note(a, self._event())

    def _fetch_stream(self):
        if self._fetch_side is None:
            self._fetch_side = torch.cuda.Stream(device=self.model._table_state.param.device)
        return self._fetch_side

    def _fetch_issue(self, k, st, block=True):
        """Send micro-batch k's requested rows (own communicator): read its
        counts (``block=False``: only if they are on the host already) and
        issue the uneven all-to-all on the fetch stream, which waits only
        for k's gather.  Returns whether k's rows are in flight."""
        f = st["fetch"][k]
        if f is None or "got" in f:
            return True
        if f["counted"] is not None:
            if not block and not f["counted"].query():
                return False
            f["counted"].synchronize()
        sc, rc = f["host"][0].tolist(), f["host"][1].tolist()
        if max(sc + rc) > f["cap"]:
            raise RuntimeError("read-set routing: an owner count above the block capacity")
        p = self.model._table_state.param
        f["need"] = f["buf"][:sum(sc)]
        rows = f["out"][:sum(rc)]
        shape = (f["need"].numel(), p.shape[1])
        self.last_exchange_bytes += f["need"].numel() * p.shape[1] * p.element_size()
        if f["gathered"] is None:  # (host tensors: no streams)
            f["got"] = torch.empty(shape, dtype=p.dtype, device=p.device)
            f["work"] = self._a2a_async(f["got"], rows, sc, rc, group=self._fetch_group)
            return True
        side = self._fetch_stream()
        with torch.cuda.stream(side):
            side.wait_event(f["gathered"])
            # allocated on the fetch stream: a block the current stream
            # freed may still be in use by its queued kernels, which this
            # stream does not wait for
            f["got"] = torch.empty(shape, dtype=p.dtype, device=p.device)
            f["work"] = self._a2a_async(f["got"], rows, sc, rc, group=self._fetch_group)
        rows.record_stream(side)
        return True

    @torch.no_grad()
    def _fetch_wait(self, k, st):
        """Before micro-batch k's forward: its rows installed (the current
        stream waits for their transfer), and k + 1's rows sent if their
        counts are on the host already (else after k's backward is issued,
        _route_chunk — the host never waits while the device idles)."""
        if not st["fetch"]:
            return
        f = st["fetch"][k]
        self._fetch_issue(k, st)  # (issued by now but for a count read that was not ready)
        a = self._event()
        if f["work"] is not None:
            f["work"].wait()
        if f["gathered"] is not None:
            torch.cuda.current_stream().wait_stream(self._fetch_stream())
        self._note(a, self._event())
        scatter_rows(self.model._table_state.param.data, f["need"], f["got"])
        if f["gathered"] is not None:  # (read here, allocated on the fetch stream)
            f["got"].record_stream(torch.cuda.current_stream())
        if k + 1 < len(st["fetch"]):
            self._fetch_issue(k + 1, st, block=False)  # in flight while micro-batch k computes
        st["fetch"][k] = None

    @torch.no_grad()
    def _route_chunk(self, k, st):
        """After micro-batch k's backward: export its table-gradient rows on
        the device (no host sync, export_stamped), then send micro-batch
        k - 1's — whose counts are ready by now, while k computes — so the
        host never waits for the micro-batch it has just issued."""
        if st["fetch"] and k + 1 < len(st["fetch"]):
            self._fetch_issue(k + 1, st)  # (if _fetch_wait(k) found its counts not ready)
        tg = self.model._tg
        rows, vals, counts, self._sr_ws = export_stamped(tg, self.world, self._sr_ws)
        ev = torch.cuda.Event()
        ev.record()
        st["export"].append((rows, vals, counts, ev))
        st["coef"] = tg.coef.clone() if st.get("coef") is None else st["coef"] + tg.coef
        tg.pending = False
        if k > 0:
            self._route_issue(k - 1, st)

    def _side(self):
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(device=self.model._table_state.param.device)
        return self._side_stream

    @torch.no_grad()
    def _route_issue(self, j, st):
        """Send micro-batch j's exported rows to their owners: on a side
        stream that waits only for j's export, so the count exchange's host
        read does not wait for the micro-batch computing meanwhile, and the
        rows' all-to-all overlaps it."""
        rows, vals, counts, ev = st["export"][j]
        st["export"][j] = None
        if not self.distributed:
            n = int(counts[0])
            st["route"].append((rows[:n], vals[:n], [n], None, None))
            return
        p = self.model._table_state.param
        d = p.shape[1]
        side = self._side()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            a = self._event()
            send = counts[1:].long()
            recv = torch.empty_like(send)
            _a2a(recv, send, group=self.group)
            sc, rc = send.tolist(), recv.tolist()
            n = sum(sc)
            rid = torch.empty(int(sum(rc)), dtype=torch.int32, device=p.device)
            _a2a(rid, rows[:n], rc, sc, group=self.group)
            self._note(a, self._event())
            rv = torch.empty(rid.numel(), d, dtype=vals.dtype, device=p.device)
            work = self._a2a_async(rv, vals[:n], rc, sc)  # in flight while j + 1 computes
        st["route"].append((rid, rv, rc, work, (rows, vals)))
        self.last_exchange_bytes += (sum(rc) - rc[self.rank]) * (4 + d * p.element_size())

    @torch.no_grad()
    def _finish_routed(self, st):
        W = self.world
        if st["export"] and st["export"][-1] is not None:
            self._route_issue(len(st["export"]) - 1, st)
        a = self._event()
        cur = torch.cuda.current_stream()
        for rid, rv, _, work, _ in st["route"]:
            if work is not None:
                work.wait()
            if self.distributed:  # allocated on the side stream, read here
                rid.record_stream(cur)
                rv.record_stream(cur)
        if self.distributed and self._side_stream is not None:
            cur.wait_stream(self._side_stream)
        self._note(a, self._event())
        blocks = [(rid, rv, counts) for rid, rv, counts, _, _ in st["route"]]
        own = torch.empty(2, device=self.model._table_state.param.device)
        self._owner_adam(blocks, self._union_coef(st["coef"]), norms=own)
        sq = own * own
        allp = torch.empty(W, 2, device=own.device)
        if self.distributed:
            a = self._event()
            dist.all_gather_into_tensor(allp.view(-1), sq, group=self.group)
            self._note(a, self._event())
        else:
            allp.copy_(sq.view(1, 2))
        tot = allp[0].clone()
        for q in range(1, W):
            tot += allp[q]
        self._norms_next = tot.sqrt()
        if self.distributed and W > 1:
            self.model.table_stale = True

    def _pipelined_step(self, users, pos, neg):
        st = {"fetch": [], "export": [], "route": [], "coef": None}

        def chunk_hook(k, phase):
            if phase == "pre":
                self._fetch_wait(k, st)
            else:
                self._route_chunk(k, st)
        tg = self.model._tg
        tg.rows_parts = self.world  # each micro-batch's S packed per owner (export_stamped)
        try:
            return self.model.stageOne(users, pos, neg, grad_hook=lambda: self._allreduce(st),
                                       loss_scale=1.0 / self.world,
                                       tree_hook=lambda trees: self._plan_fetch(trees, st),
                                       chunks=self.microbatches, chunk_hook=chunk_hook)
        finally:
            tg.rows_parts = None
            tg.export = None

    @torch.no_grad()
    def sync_table(self):
        """``fetch``: all-gather the owners' row blocks, so every rank's table
        is current everywhere (before inference or a checkpoint)."""
        if self.table_exchange != "fetch" or not self.distributed:
            return
        p = self.model._table_state.param
        N, d = p.shape
        n_own = N // self.world
        lo = self.rank * n_own
        pf = p.data.view(-1)
        dist.all_gather_into_tensor(pf, pf[lo * d:(lo + n_own) * d].clone(), group=self.group)
        self.model.table_stale = False

    def gather_optimizer_state(self):
        """All-gather the row shards of the sharded parameters' Adam moments
        (for a checkpoint: afterwards every rank holds the full state) and,
        under ``fetch``, the table itself (sync_table)."""
        if not self.distributed:
            return
        self.sync_table()
        for st in self._states.values():
            if id(st.param) in self._sharded:
                for t in (st.exp_avg, st.exp_avg_sq):
                    f = t.view(-1)
                    n = f.numel() // self.world
                    dist.all_gather_into_tensor(f, f[self.rank * n:(self.rank + 1) * n].clone(),
                                                group=self.group)
                st.stale_rows = False

    def _allreduce(self, pipelined: dict | None = None):
        if pipelined is not None:  # the micro-batches' routed rows: owner Adam
            self._finish_routed(pipelined)
        if not self.distributed:
            return
        tg = getattr(self.model, "_tg", None)
        if (pipelined is None and self.table_exchange != "dense" and tg is not None
                and tg.pending):
            self._routed_table_step()
        params = [p for p in self.model.parameters() if p.grad is not None]
        # large gradients (the id tables) are reduced in place or by row shard;
        # the small ones share one flattened bucket
        big = [p for p in params if p.grad.numel() >= self.BUCKET_MIN and p.grad.is_contiguous()]
        small = [p.grad for p in params
                 if not (p.grad.numel() >= self.BUCKET_MIN and p.grad.is_contiguous())]
        for p in big:
            if self._shardable(p):
                self._sharded_adam(p)
            else:
                a = self._event()
                dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group)
                self._note(a, self._event())
                self.last_exchange_bytes += 2 * (self.world - 1) * p.grad.numel() \
                    * p.grad.element_size() // self.world
        if small:
            flat = torch.cat([g.reshape(-1) for g in small])
            a = self._event()
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            self._note(a, self._event())
            self.last_exchange_bytes += 2 * (self.world - 1) * flat.numel() * 4 // self.world
            off = 0
            for g in small:
                g.copy_(flat[off: off + g.numel()].view_as(g))
                off += g.numel()

    def table_stepped_by_hook(self) -> bool:
        """Whether the exchange hook itself steps the id table (routed
        exchange, or the row-sharded dense Adam of a large table)."""
        st = getattr(self.model, "_table_state", None)
        if st is None:
            return False
        if self.table_exchange != "dense":
            return True
        p = st.param
        return (self.world > 1 and self.shard_optimizer and p.numel() >= self.BUCKET_MIN
                and p.shape[0] % self.world == 0)

    def step(self, users, pos, neg):
        self.last_exchange_bytes = 0
        if self.table_exchange == "fetch" and self.microbatches > 1:
            return self._pipelined_step(users, pos, neg)
        kw = {}
        if self.table_exchange == "fetch":
            kw["tree_hook"] = self.fetch_rows
        if getattr(self.model, "captures_dp_step", False):
            # SASRec: the captured step, split around this exchange
            kw["table_by_hook"] = self.table_stepped_by_hook()
        return self.model.stageOne(users, pos, neg, grad_hook=self._allreduce,
                                   loss_scale=1.0 / self.world, **kw)
