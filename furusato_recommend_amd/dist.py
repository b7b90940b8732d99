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
Both give the gradient of the union batch; replicas stay bit-identical.

The initial parameters are broadcast from rank 0 (the DDP ctor broadcast,
ddp_lgcn.py:663).  The engine is duck-typed (forward / bpr / backward /
adam_step), so the CPU tests drive this exact driver with gloo and an
oracle-backed engine.  The forward is frontier-pruned to the rank's own
batch; after the sparse exchange the backward is pruned to the union seeds.
"""
from __future__ import annotations

import datetime
import os

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


class DataParallel:
    def __init__(self, engine, emb: torch.Tensor, adam, group=None, mode: str = "sparse"):
        if mode not in ("sparse", "dense"):
            raise ValueError(mode)
        self.mode = mode
        self.engine = engine
        self.emb = emb
        self.adam = adam
        self.group = group
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.grad = torch.empty_like(emb) if mode == "dense" else None
        if self.world > 1:
            dist.broadcast(emb.data, src=0, group=group)

    def shard(self):
        """(shard, n_shards) for the on-device sampler."""
        return self.rank, self.world

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

    def step(self, users, pos, neg, decay: float, loss_accum=None):
        eng = self.engine
        out = eng.forward_for_batch(self.emb, users, pos, neg)
        loss = eng.bpr(out, self.emb, users, pos, neg, decay, loss_accum,
                       grad_scale=1.0 / self.world)
        if self.mode == "sparse":
            keys, rows_p, rows_e = eng.export_seeds()
            if self.distributed:
                keys, rows_p, rows_e = self._exchange(keys, rows_p, rows_e)
            eng.import_seeds(keys, rows_p, rows_e)
            eng.backward(self.emb, adam=self.adam)
        else:
            eng.backward(self.emb, grad_out=self.grad)
            if self.distributed:
                dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.group)
            eng.adam_step(self.emb, self.grad, self.adam)
        return loss


class DenseGradDataParallel:
    """Data parallelism for models trained through autograd (GraphSAGE;
    replaces ddp_sage.py:754-878, which like ddp_lgcn.py never synchronised
    gradients).  Every rank samples its own user shard; the loss is scaled by
    1/world_size and the gradients of all parameters are SUM-all-reduced over
    RCCL as one flattened bucket between backward and the (HIP) Adam step."""

    BUCKET_MIN = 1 << 20  # elements: gradients this large are reduced in place

    def __init__(self, model, group=None):
        self.model = model
        self.group = group
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        tg = getattr(model, "_tg", None)
        if tg is not None and self.world > 1:
            # GraphSAGE's sorted table gradient: materialise it as .grad so it
            # can be all-reduced (the fused table Adam needs the local S only)
            tg.dense = True
        if self.world > 1:
            for p in model.parameters():
                dist.broadcast(p.data, src=0, group=group)

    def _allreduce(self):
        if not self.distributed:
            return
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        # large gradients (the id table) are reduced in place; the small ones
        # share one flattened bucket
        big = [g for g in grads if g.numel() >= self.BUCKET_MIN and g.is_contiguous()]
        small = [g for g in grads if not (g.numel() >= self.BUCKET_MIN and g.is_contiguous())]
        for g in big:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
        if small:
            flat = torch.cat([g.reshape(-1) for g in small])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            off = 0
            for g in small:
                g.copy_(flat[off: off + g.numel()].view_as(g))
                off += g.numel()

    def step(self, users, pos, neg):
        return self.model.stageOne(users, pos, neg, grad_hook=self._allreduce,
                                   loss_scale=1.0 / self.world)
