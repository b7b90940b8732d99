"""Top-k ranking metrics with the reference's exact semantics.

utils.py:40-48 (getLabel), metric.py:60-103 (RecallPrecision_ATk, NDCGatK_r):
recall sums hits/(|gt| + 1e-6) per user, precision sums hits/k, NDCG uses the
binary-relevance DCG with an ideal DCG over min(k, |gt|) positions.  Sums are
per batch; the caller divides by the number of evaluated users
(trainer.py:166-170).
"""
from __future__ import annotations

import numpy as np


def getLabel(test_data, pred_data) -> np.ndarray:
    r = np.zeros((len(test_data), pred_data.shape[1] if len(test_data) else 0))
    for i, gt in enumerate(test_data):
        r[i] = np.isin(pred_data[i], np.asarray(list(gt)))
    return r.astype("float")


def RecallPrecision_ATk(test_data, r, k):
    right_pred = r[:, :k].sum(1)
    recall_n = np.array([len(test_data[i]) for i in range(len(test_data))])
    recall = np.sum(right_pred / (recall_n + 1e-6))
    precis = np.sum(right_pred) / k
    hr = np.sum(right_pred >= 1)
    return {"recall": recall, "precision": precis, "hr": hr}


def NDCGatK_r(test_data, r, k):
    assert len(r) == len(test_data)
    pred_data = r[:, :k]
    test_matrix = np.zeros((len(pred_data), k))
    for i, items in enumerate(test_data):
        length = k if k <= len(items) else len(items)
        test_matrix[i, :length] = 1
    idcg = np.sum(test_matrix * 1.0 / np.log2(np.arange(2, k + 2)), axis=1)
    dcg = np.sum(pred_data * (1.0 / np.log2(np.arange(2, k + 2))), axis=1)
    idcg[idcg == 0.0] = 1.0
    ndcg = dcg / idcg
    ndcg[np.isnan(ndcg)] = 0.0
    return np.sum(ndcg)


def test_one_batch(sorted_items: np.ndarray, groundTrue, topks=(10, 20)) -> dict:
    """trainer.py:263-280 without the proprietary-data Diversity term."""
    r = getLabel(groundTrue, sorted_items)
    out = {"recall": [], "precision": [], "ndcg": [], "hr": []}
    for k in topks:
        ret = RecallPrecision_ATk(groundTrue, r, k)
        out["precision"].append(ret["precision"])
        out["recall"].append(ret["recall"])
        out["hr"].append(ret["hr"])
        out["ndcg"].append(NDCGatK_r(groundTrue, r, k))
    return {k: np.array(v) for k, v in out.items()}
