"""MF-BPR (model/MF.py:35-112) on the same HIP engine.

Matrix factorisation is LightGCN with zero propagation layers: scores are
dot products of the ego embeddings and the reg term is taken on the same
rows.  The two reference tables ``embedding_user`` / ``embedding_item`` are
views into one [n_users + m_items, d] device table so the fused BPR /
seed / Adam kernels (one pass over the table) serve both; ``state_dict``
keeps the reference keys ``embedding_user.weight`` / ``embedding_item.weight``.

``device="cpu"`` is configuration C1 as BASELINE states it ("CPU
single-process, no GPU"): the same model on host arrays, stepped by the
library's host code — mirec_cpu_bpr_sample (the device sampler's streams on
CPU threads: the same triples) and mirec_cpu_bpr_step (BPR loss, backward,
dense Adam) — and evaluated with the reference's own rating / mask / topk
arithmetic on the CPU (trainer.py:115-138).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

from ._lib import check, lib, ptr
from .engine import AdamState, PropagationEngine
from .graph import DEFAULT_SPLIT, Graph, positive_probs


class MF(nn.Module):
    def __init__(self, config: dict, dataset):
        super().__init__()
        self.config = config
        self.num_users = int(dataset.n_users)
        self.num_items = int(dataset.m_items)
        self.latent_dim = int(config.get("latent_dim_rec", config.get("recdim", 32)))
        self.device = torch.device(config.get("device", "cuda:0"))
        if self.device.type not in ("cuda", "cpu"):
            raise RuntimeError(f"MF (furusato_recommend_amd): no {self.device.type} path")
        self.on_host = self.device.type == "cpu"
        # model/MF.py:47-54: default nn.Embedding init, N(0, 1)
        table = torch.randn(self.num_users + self.num_items, self.latent_dim,
                            device=self.device)
        self._table = table
        self.embedding_user = nn.Embedding(self.num_users, self.latent_dim,
                                           _weight=table[: self.num_users], device=self.device)
        self.embedding_item = nn.Embedding(self.num_items, self.latent_dim,
                                           _weight=table[self.num_users:], device=self.device)
        self.f = nn.Sigmoid()
        self.graph = Graph.from_interactions(dataset.trainUser, dataset.trainItem,
                                             self.num_users, self.num_items, self.device,
                                             split=int(config.get("csr_split", DEFAULT_SPLIT)))
        self.graph.set_positive_probs(positive_probs(config))
        self.optim = AdamState(self._table, lr=config["lr"])
        self._loss_accum = torch.zeros(1, dtype=torch.float32, device=self.device)
        if self.on_host:
            self.engine = None
            self._grad_ws = torch.empty_like(self._table)
            self.n_threads = int(config.get("n_threads", os.cpu_count() or 1))
        else:
            self.engine = PropagationEngine(self.graph, self.latent_dim, 0,
                                            int(config.get("bpr_batch_size", 2048)))

    def load_table(self, user_w: torch.Tensor, item_w: torch.Tensor):
        with torch.no_grad():
            self._table[: self.num_users].copy_(user_w)
            self._table[self.num_users:].copy_(item_w)

    @torch.no_grad()
    def getUsersRating(self, users):
        users_emb = self.embedding_user.weight[users.long()]
        return self.f(users_emb @ self.embedding_item.weight.t())

    @torch.no_grad()
    def eval_ratings(self):
        """users -> sigmoid(U Iᵀ) rows (model/MF.py:56-60)."""
        items = self.embedding_item.weight
        return lambda users: self.f(self.embedding_user.weight[users.long()] @ items.t())

    @torch.no_grad()
    def propagated(self) -> torch.Tensor:
        return self._table

    def eval_embeddings(self):
        """(user rows, item rows): the operands of the streaming evaluation
        (evaluate.score_topk).  The reference ranks sigmoid(U Iᵀ)
        (model/MF.py:56-60); sigmoid is monotone, so the top-k of the raw
        scores is a top-k of the ratings — where fp32 sigmoid saturates to
        equal values, torch.topk may break the tie either way and the raw
        score breaks it here."""
        return self._table[: self.num_users], self._table[self.num_users:]

    def sample(self, n_triples: int, seed: int, offset: int = 0, shard: int = 0,
               n_shards: int = 1):
        """UniformSample (negative_sample.py:98-134) on the model's device:
        int32 (users, pos, neg) tensors (on the host: the device sampler's
        streams, the same triples)."""
        from .engine import sample_triples
        u = torch.empty(n_triples, dtype=torch.int32, device=self.device)
        p, n = torch.empty_like(u), torch.empty_like(u)
        err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if self.on_host:
            g = self.graph
            check(lib.mirec_cpu_bpr_sample(
                g.rowptr_host.ctypes.data, g.col_host.ctypes.data, ptr(g.col_sorted),
                ptr(getattr(g, "pos_cdf", None)), g.n_users, g.m_items, int(n_triples),
                ctypes.c_uint64(seed & (2**64 - 1)), ctypes.c_uint64(offset & (2**64 - 1)),
                int(shard), int(n_shards), u.data_ptr(), p.data_ptr(), n.data_ptr(),
                err.data_ptr(), self.n_threads), "cpu_bpr_sample")
        else:
            sample_triples(self.graph, n_triples, seed, offset, u, p, n, err, shard, n_shards)
        self._sample_err = err
        return u, p, n

    def bpr_loss(self, users, pos, neg):
        users_emb = self.embedding_user(users.long())
        pos_emb = self.embedding_item(pos.long())
        neg_emb = self.embedding_item(neg.long())
        pos_scores = torch.sum(users_emb * pos_emb, dim=1)
        neg_scores = torch.sum(users_emb * neg_emb, dim=1)
        loss = torch.mean(nn.functional.softplus(neg_scores - pos_scores))
        reg = 0.5 * (users_emb.norm(2).pow(2) + pos_emb.norm(2).pow(2)
                     + neg_emb.norm(2).pow(2)) / float(len(users))
        return loss, reg

    def forward(self, users, items):
        u = self.embedding_user(users.long())
        i = self.embedding_item(items.long())
        return self.f(torch.sum(u * i, dim=1))

    def _as_i32(self, t):
        t = torch.as_tensor(t)
        return t.to(device=self.device, dtype=torch.int32).contiguous()

    @torch.no_grad()
    def stageOne(self, user, pos, neg, loss_accum=None):
        if self.on_host:
            return self._host_step(self._as_i32(user), self._as_i32(pos), self._as_i32(neg),
                                   loss_accum)
        return self.engine.train_step(self._table, self.optim, self._as_i32(user),
                                      self._as_i32(pos), self._as_i32(neg),
                                      float(self.config["decay"]), loss_accum).clone()

    def _host_step(self, u, p, n, loss_accum=None):
        """model/MF.py:88-94 on the host (mirec_cpu_bpr_step)."""
        hp = self.optim.next_hparams()
        out = ctypes.c_float(0.0)
        st = self.optim
        check(lib.mirec_cpu_bpr_step(self._table.data_ptr(), st.exp_avg.data_ptr(),
                                     st.exp_avg_sq.data_ptr(), self._grad_ws.data_ptr(),
                                     self._table.shape[0], self.latent_dim, self.num_users,
                                     u.data_ptr(), p.data_ptr(), n.data_ptr(), u.numel(),
                                     float(self.config["decay"]), ctypes.byref(hp),
                                     ctypes.byref(out), self.n_threads), "cpu_bpr_step")
        loss = torch.tensor(out.value, dtype=torch.float32)
        if loss_accum is not None:
            loss_accum += loss
        return loss

    def host_grad(self, u, p, n, grad_scale: float = 1.0):
        """The gradient half of the host step (mirec_cpu_bpr_grad): dLoss/dtable
        of one batch x ``grad_scale`` into ``self.host_grad_buffer``; returns
        the (unscaled) loss.  With host_adam: dist.HostDataParallel's step."""
        u, p, n = self._as_i32(u), self._as_i32(p), self._as_i32(n)
        out = ctypes.c_float(0.0)
        check(lib.mirec_cpu_bpr_grad(self._table.data_ptr(), self._grad_ws.data_ptr(),
                                     self._table.shape[0], self.latent_dim, self.num_users,
                                     u.data_ptr(), p.data_ptr(), n.data_ptr(), u.numel(),
                                     float(self.config["decay"]), float(grad_scale),
                                     ctypes.byref(out), self.n_threads), "cpu_bpr_grad")
        return torch.tensor(out.value, dtype=torch.float32)

    @property
    def host_grad_buffer(self) -> torch.Tensor:
        return self._grad_ws

    def host_adam(self):
        """Adam over the whole table from ``host_grad_buffer`` (mirec_cpu_adam)."""
        hp = self.optim.next_hparams()
        st = self.optim
        check(lib.mirec_cpu_adam(self._table.data_ptr(), self._grad_ws.data_ptr(),
                                 st.exp_avg.data_ptr(), st.exp_avg_sq.data_ptr(),
                                 self._table.numel(), ctypes.byref(hp), self.n_threads),
              "cpu_adam")

    @torch.no_grad()
    def OneEpoch(self, user, pos, neg):
        B = int(self.config["bpr_batch_size"])
        n = len(user)
        user, pos, neg = self._as_i32(user), self._as_i32(pos), self._as_i32(neg)
        self._loss_accum.zero_()
        for i in range(0, n, B):
            if self.on_host:
                self._host_step(user[i:i + B], pos[i:i + B], neg[i:i + B], self._loss_accum)
                continue
            self.engine.train_step(self._table, self.optim, user[i:i + B], pos[i:i + B],
                                   neg[i:i + B], float(self.config["decay"]),
                                   self._loss_accum)
        return self._loss_accum[0] / (n // B + 1)
