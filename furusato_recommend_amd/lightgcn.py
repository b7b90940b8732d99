"""LightGCN with the reference's model-class surface, on the HIP engine.

Drop-in for ``model.lgcn.LightGCN`` (model/lgcn.py:44-151): same constructor
``(config, dataset)``, same methods (``forward``, ``getEmbedding``,
``bpr_loss``, ``getUsersRating``, ``stageOne``, ``OneEpoch``) and the same
``state_dict`` key ``all_embedding.weight`` [(n_users + m_items), recdim], so
reference checkpoints load unchanged.

Two execution paths, both on libmirec:
  * ``stageOne`` / ``OneEpoch`` — the training hot path: the fused engine
    step (engine.PropagationEngine.train_step), no autograd graph, Adam fused
    into the last backward layer.
  * ``forward`` / ``bpr_loss`` — differentiable: propagation is an
    autograd.Function whose backward is the same HIP SpMM (Â is symmetric),
    for callers that build their own loss.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .engine import AdamState, PropagationEngine, sample_triples
from .graph import DEFAULT_SPLIT, Graph, positive_probs


class _Propagate(torch.autograd.Function):
    """out = (Σ_{l=0..L} Â^l E)/(L+1) with a HIP backward (Horner, dense seed)."""

    @staticmethod
    def forward(ctx, emb, engine: PropagationEngine):
        ctx.engine = engine
        return engine.forward(emb.contiguous()).clone()

    @staticmethod
    def backward(ctx, grad_out):
        eng = ctx.engine
        L = eng.L
        d = (grad_out.contiguous() / float(L + 1))
        if L == 0:
            return d, None
        g = d
        for _ in range(L):
            nxt = torch.empty_like(d)
            eng.propagate_accumulate(g, d, nxt)
            g = nxt
        return g, None


def _config_get(config, *keys, default=None):
    for k in keys:
        if k in config:
            return config[k]
    return default


class LightGCN(nn.Module):
    """model/lgcn.py:44-151 on MI355X."""

    def __init__(self, config: dict, dataset):
        super().__init__()
        self.dataset = dataset
        self.config = config
        self.num_users = int(dataset.n_users)
        self.num_items = int(dataset.m_items)
        self.latent_dim = int(_config_get(config, "recdim", "latent_dim_rec", default=64))
        self.num_layers = int(_config_get(config, "layer", "lightGCN_n_layers", default=3))
        self.device = torch.device(config.get("device", "cuda:0"))
        if self.device.type != "cuda":
            raise RuntimeError("LightGCN (furusato_recommend_amd) runs on a HIP device only")
        self.graph = Graph.from_interactions(dataset.trainUser, dataset.trainItem,
                                             self.num_users, self.num_items, self.device,
                                             split=int(config.get("csr_split", DEFAULT_SPLIT)))
        self.graph.set_positive_probs(positive_probs(config))
        self.__init_weight()
        self.optim = AdamState(self.all_embedding.weight, lr=config["lr"])
        self.engine = PropagationEngine(self.graph, self.latent_dim, self.num_layers,
                                        int(config.get("bpr_batch_size", 2048)),
                                        prune=bool(config.get("prune", True)))
        self._loss_accum = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.test_item_emb = None

    def __init_weight(self):
        # model/lgcn.py:70-76: Embedding(n_items + n_users, d), N(0, 0.1)
        self.all_embedding = nn.Embedding(self.num_items + self.num_users, self.latent_dim,
                                          device=self.device)
        nn.init.normal_(self.all_embedding.weight, std=0.1)

    # --------------------------------------------------------- reference API
    def forward(self):
        out = _Propagate.apply(self.all_embedding.weight, self.engine)
        return out[: self.num_users], out[self.num_users:]

    def getEmbedding(self, users, pos_items, neg_items):
        all_users, all_items = self.forward()
        users_emb = all_users[users]
        pos_emb = all_items[pos_items]
        neg_emb = all_items[neg_items]
        users_emb_ego = self.all_embedding(users)
        pos_emb_ego = self.all_embedding(pos_items + self.num_users)
        neg_emb_ego = self.all_embedding(neg_items + self.num_users)
        return users_emb, pos_emb, neg_emb, users_emb_ego, pos_emb_ego, neg_emb_ego

    def bpr_loss(self, users, pos, neg):
        (users_emb, pos_emb, neg_emb, userEmb0, posEmb0, negEmb0) = self.getEmbedding(
            users.long(), pos.long(), neg.long())
        reg_loss = (0.5 * (userEmb0.norm(2).pow(2) + posEmb0.norm(2).pow(2)
                           + negEmb0.norm(2).pow(2)) / float(len(users)))
        pos_scores = torch.sum(users_emb * pos_emb, dim=1)
        neg_scores = torch.sum(users_emb * neg_emb, dim=1)
        loss = torch.mean(torch.nn.functional.softplus(neg_scores - pos_scores))
        return loss, reg_loss

    @torch.no_grad()
    def propagated(self) -> torch.Tensor:
        """Full layer-mean embeddings [N, D] (no autograd; the engine's
        buffer, valid until the next engine call).  Propagates only when the
        table changed since the last full propagation."""
        return self.engine.forward_cached(self.all_embedding.weight)

    @torch.no_grad()
    def getUsersRating(self, users):
        """model/lgcn.py:120-125.  The reference re-propagates the whole graph
        on every call — once per 10 000-user batch of Trainer.test
        (trainer.py:130); here the propagation is reused while the table is
        unchanged, so an unchanged reference Trainer.test propagates once
        per evaluation."""
        out = self.propagated()
        users_emb = out[users.long()]
        items_emb = out[self.num_users:]
        return torch.matmul(users_emb, items_emb.t())

    @torch.no_grad()
    def eval_ratings(self):
        """users -> rating rows [len(users), m_items] with ONE propagation for
        the whole evaluation (getUsersRating semantics, model/lgcn.py:120-125)."""
        out = self.propagated()
        items = out[self.num_users:]
        return lambda users: out[users.long()] @ items.t()

    def eval_embeddings(self):
        """(user rows [n_users, D], item rows [m_items, D]) of one propagation:
        the operands of the streaming evaluation (evaluate.score_topk)."""
        out = self.propagated()
        return out[: self.num_users], out[self.num_users:]

    def _as_i32(self, t):
        if not torch.is_tensor(t):
            t = torch.as_tensor(t)
        return t.to(device=self.device, dtype=torch.int32, non_blocking=True).contiguous()

    @torch.no_grad()
    def stageOne(self, user, pos, neg, loss_accum=None):
        """One fused BPR step (model/lgcn.py:127-133); returns the loss tensor."""
        w = self.all_embedding.weight
        return self.engine.train_step(w, self.optim, self._as_i32(user), self._as_i32(pos),
                                      self._as_i32(neg), float(self.config["decay"]),
                                      loss_accum).clone()

    @torch.no_grad()
    def OneEpoch(self, user, pos, neg):
        """model/lgcn.py:135-151: minibatch loop; mean loss over len//B + 1."""
        B = int(self.config["bpr_batch_size"])
        n = len(user)
        total_batch = n // B + 1
        user, pos, neg = self._as_i32(user), self._as_i32(pos), self._as_i32(neg)
        self._loss_accum.zero_()
        for i in range(0, n, B):
            self.engine.train_step(self.all_embedding.weight, self.optim, user[i:i + B],
                                   pos[i:i + B], neg[i:i + B], float(self.config["decay"]),
                                   self._loss_accum)
        return self._loss_accum[0] / total_batch

    # ------------------------------------------------------------- sampling
    def sample(self, n_triples: int, seed: int, offset: int = 0, shard: int = 0,
               n_shards: int = 1):
        """On-device UniformSample: int32 (users, pos, neg) device tensors."""
        dev = self.device
        u = torch.empty(n_triples, dtype=torch.int32, device=dev)
        p = torch.empty_like(u)
        n = torch.empty_like(u)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        sample_triples(self.graph, n_triples, seed, offset, u, p, n, err, shard, n_shards)
        self._sample_err = err
        return u, p, n

    def optimizer_state_dict(self):
        return self.optim.state_dict()
