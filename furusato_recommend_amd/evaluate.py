"""Recall@k / NDCG@k evaluation (Trainer.test, trainer.py:115-187).

The layer-mean embeddings are propagated ONCE per evaluation with the HIP
engine (the reference re-propagates per 10 000-user batch through
getUsersRating, model/lgcn.py:120-125).  Per batch of users:
rating = U_b · Iᵀ (library GEMM, hipBLASLt via torch.matmul, as the
reference's torch.matmul), then one HIP launch (mirec_topk_masked) sets the
user's train positives to -1024 in place (trainer.py:132-137) and selects the
top-k (trainer.py:138); metric sums on the host with the reference formulas
(metric.py:60-103).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .metric import test_one_batch


@torch.no_grad()
def topk_masked(rating: torch.Tensor, users: torch.Tensor, graph, k: int,
                mask: bool = True):
    """In-place mask of train positives + top-k of each rating row (HIP)."""
    if rating.dtype != torch.float32 or not rating.is_contiguous():
        raise ValueError("rating must be contiguous float32")
    n_eval, m = rating.shape
    users = users.to(torch.int32).contiguous()
    idx = torch.empty(n_eval, k, dtype=torch.int32, device=rating.device)
    val = torch.empty(n_eval, k, dtype=torch.float32, device=rating.device)
    check(lib.mirec_topk_masked(rating.data_ptr(), n_eval, m, users.data_ptr(),
                                graph.csr_ptr() if mask else None, graph.n_users, int(k),
                                idx.data_ptr(), val.data_ptr(), _lib.stream_handle()),
          "topk_masked")
    return val, idx


@torch.no_grad()
def evaluate(model, test_dict: dict, topks=(10, 20), batch: int = 10000,
             return_topk: bool = False):
    users = np.array(sorted(test_dict.keys()), dtype=np.int64)
    res = {m: np.zeros(len(topks)) for m in ("precision", "recall", "ndcg", "hr")}
    if users.size == 0:
        return res
    ratings = model.eval_ratings()   # propagates once, returns users -> rating rows
    kmax = max(topks)
    tops = []
    for i in range(0, len(users), batch):
        bu = torch.from_numpy(users[i:i + batch]).to(model.device)
        rating = ratings(bu).contiguous()
        _, top = topk_masked(rating, bu, model.graph, kmax)
        top = top.cpu().numpy()
        if return_topk:
            tops.append(top)
        gt = [test_dict[int(u)] for u in users[i:i + batch]]
        r = test_one_batch(top, gt, topks)
        for m in res:
            res[m] += r[m]
    for m in res:
        res[m] /= float(len(users))
    if return_topk:
        return res, np.concatenate(tops)
    return res
