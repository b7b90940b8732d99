"""Recall@k / NDCG@k evaluation (Trainer.test, trainer.py:115-187).

The layer-mean embeddings are propagated ONCE per evaluation with the HIP
engine (the reference re-propagates per 10 000-user batch through
getUsersRating, model/lgcn.py:120-125).  Per batch of users, for a model
with ``eval_embeddings`` (LightGCN, MF) and k <= 32: mirec_score_topk streams
the scores U_b · Iᵀ through MFMA tiles straight into per-user top-k
candidates, the train positives at -1024 (trainer.py:132-138) — the
[batch, M] rating matrix is never written (MF's sigmoid ratings rank like
its raw scores: sigmoid is monotone).  Otherwise (k > 32, or a width
outside STREAM_DIMS): rating = U_b · Iᵀ (library GEMM, as the reference's
torch.matmul), then mirec_topk_masked masks in place and selects.  Metric
sums on the host with the reference formulas (metric.py:60-103).
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


STREAM_DIMS = (16, 32, 64, 128, 256)
STREAM_MAX_K = 32


@torch.no_grad()
def score_topk(user_rows: torch.Tensor, items: torch.Tensor, users: torch.Tensor, graph,
               k: int, mask: bool = True):
    """Top-k of user_rows · itemsᵀ per row with the users' train positives
    at -1024, streamed (mirec_score_topk): (values, item ids) [n, k]."""
    n, d = user_rows.shape
    user_rows, items = user_rows.contiguous(), items.contiguous()
    users = users.to(torch.int32).contiguous()
    idx = torch.empty(n, k, dtype=torch.int32, device=user_rows.device)
    val = torch.empty(n, k, dtype=torch.float32, device=user_rows.device)
    ws = torch.empty(max(int(lib.mirec_score_topk_workspace(n, items.shape[0], k)), 1),
                     dtype=torch.uint8, device=user_rows.device)
    check(lib.mirec_score_topk(user_rows.data_ptr(), n, items.data_ptr(), items.shape[0], d,
                               users.data_ptr(), graph.csr_ptr() if mask else None,
                               graph.n_users, int(k), idx.data_ptr(), val.data_ptr(),
                               ws.data_ptr(), ws.numel(), _lib.stream_handle()), "score_topk")
    return val, idx


@torch.no_grad()
def evaluate(model, test_dict: dict, topks=(10, 20), batch: int = 10000,
             return_topk: bool = False, stream: bool | None = None):
    users = np.array(sorted(test_dict.keys()), dtype=np.int64)
    res = {m: np.zeros(len(topks)) for m in ("precision", "recall", "ndcg", "hr")}
    if users.size == 0:
        return res
    kmax = max(topks)
    if getattr(model, "device", None) is not None and torch.device(model.device).type == "cpu":
        return _evaluate_host(model, test_dict, users, topks, batch, return_topk, res)
    emb = None
    if stream is not False and hasattr(model, "eval_embeddings") and kmax <= STREAM_MAX_K:
        emb = model.eval_embeddings()   # propagates once
        if emb[0].shape[1] not in STREAM_DIMS:
            emb = None
    if emb is None:
        ratings = model.eval_ratings()   # propagates once, returns users -> rating rows
    tops = []
    for i in range(0, len(users), batch):
        bu = torch.from_numpy(users[i:i + batch]).to(model.device)
        if emb is not None:
            _, top = score_topk(emb[0][bu], emb[1], bu, model.graph, kmax)
        else:
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


@torch.no_grad()
def _evaluate_host(model, test_dict, users, topks, batch, return_topk, res):
    """A CPU model (configuration C1): the reference's own arithmetic on the
    host — rating = model.eval_ratings() rows, the train positives set to
    -1024, torch.topk (trainer.py:115-138) — and the same metric sums."""
    kmax = max(topks)
    ratings = model.eval_ratings()
    g = model.graph
    rp, col, nu = g.rowptr_host, g.col_host, g.n_users
    tops = []
    for i in range(0, len(users), batch):
        bu = users[i:i + batch]
        rating = ratings(torch.from_numpy(bu)).clone()
        for r, u in enumerate(bu.tolist()):
            items = col[rp[u]:rp[u + 1]].astype(np.int64) - nu
            rating[r, torch.from_numpy(items[(items >= 0) & (items < rating.shape[1])])] = -1024.0
        top = torch.topk(rating, kmax).indices.numpy()
        if return_topk:
            tops.append(top)
        r_ = test_one_batch(top, [test_dict[int(u)] for u in bu], topks)
        for m in res:
            res[m] += r_[m]
    for m in res:
        res[m] /= float(len(users))
    if return_topk:
        return res, np.concatenate(tops)
    return res
