"""Recall@k / NDCG@k evaluation (Trainer.test, trainer.py:115-187).

The layer-mean embeddings are propagated ONCE per evaluation with the HIP
engine (the reference re-propagates per 10 000-user batch through
getUsersRating, model/lgcn.py:120-125).  Per batch: rating = U_b · Iᵀ,
train positives (the user's CSR row) set to -1024 (trainer.py:132-137),
top-k (:138); metric sums on the host with the reference formulas.
"""
from __future__ import annotations

import numpy as np
import torch

from .metric import test_one_batch


def _mask_train_positives(rating: torch.Tensor, users: torch.Tensor, graph) -> None:
    rp = graph.rowptr
    starts = rp[users]
    lens = rp[users + 1] - starts
    total = int(lens.sum())
    if total == 0:
        return
    row = torch.repeat_interleave(torch.arange(users.numel(), device=users.device), lens)
    first = torch.repeat_interleave(starts - (torch.cumsum(lens, 0) - lens), lens)
    pos = first + torch.arange(total, device=users.device)
    items = graph.col[pos].long() - graph.n_users
    rating[row, items] = -(1 << 10)


@torch.no_grad()
def evaluate(model, test_dict: dict, topks=(10, 20), batch: int = 10000) -> dict:
    users = np.array(sorted(test_dict.keys()), dtype=np.int64)
    if users.size == 0:
        return {m: np.zeros(len(topks)) for m in ("precision", "recall", "ndcg", "hr")}
    out = model.propagated()
    n_users = model.num_users
    user_emb, item_emb = out[:n_users], out[n_users:]
    kmax = max(topks)
    res = {m: np.zeros(len(topks)) for m in ("precision", "recall", "ndcg", "hr")}
    for i in range(0, len(users), batch):
        bu = torch.from_numpy(users[i:i + batch]).to(out.device)
        rating = user_emb[bu] @ item_emb.t()
        _mask_train_positives(rating, bu, model.graph)
        _, top = torch.topk(rating, k=kmax)
        gt = [test_dict[int(u)] for u in users[i:i + batch]]
        r = test_one_batch(top.cpu().numpy(), gt, topks)
        for m in res:
            res[m] += r[m]
    for m in res:
        res[m] /= float(len(users))
    return res
