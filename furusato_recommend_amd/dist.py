"""User-sharded data parallelism over RCCL (replaces ddp_lgcn.py:625-768).

One process per GPU (launched by torch.distributed.run).  Every rank holds a
full replica of the embedding table, the CSR and the optimizer state (C2:
282 MB per [N, D] tensor).  Per step each rank

  1. draws its own B triples on device from the users of its shard
     (u % world_size == rank; mirec_bpr_sample), so the union batch covers
     every user with no sampling collective;
  2. runs the full-graph forward / BPR / backward with its gradient seeds
     scaled by 1/world_size, writing the dense gradient dE [N, D];
  3. SUM-all-reduces dE over RCCL (xGMI), which makes it exactly the
     gradient of the union batch of world_size * B triples (the reference's
     DDP never synchronises gradients because it calls `.module.OneEpoch`,
     ddp_lgcn.py:673 — this is what it meant to do);
  4. applies the dense Adam kernel; replicas stay bit-identical because every
     rank applies the same reduced gradient to the same parameters.

The initial parameters are broadcast from rank 0 (the DDP ctor broadcast,
ddp_lgcn.py:663).  The engine is duck-typed (forward / bpr / backward /
adam_step), so the CPU tests drive this exact driver with gloo and an
oracle-backed engine.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class DataParallel:
    def __init__(self, engine, emb: torch.Tensor, adam, group=None):
        self.engine = engine
        self.emb = emb
        self.adam = adam
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.grad = torch.empty_like(emb)
        if self.world > 1:
            dist.broadcast(emb.data, src=0, group=group)

    def shard(self):
        """(shard, n_shards) for the on-device sampler."""
        return self.rank, self.world

    def step(self, users, pos, neg, decay: float, loss_accum=None):
        eng = self.engine
        out = eng.forward(self.emb)
        loss = eng.bpr(out, self.emb, users, pos, neg, decay, loss_accum,
                       grad_scale=1.0 / self.world)
        eng.backward(self.emb, grad_out=self.grad)
        if self.world > 1:
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.group)
        eng.adam_step(self.emb, self.grad, self.adam)
        return loss
