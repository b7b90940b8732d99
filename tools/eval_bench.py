"""Evaluation top-k on the C2 configuration (1 M users x 100 K items, d =
64): streamed scores (mirec_score_topk: MFMA tiles filtered into per-user
candidates, no rating matrix) vs the dense path (library GEMM writes the
[batch, M] ratings, mirec_topk_masked reads them).  One JSON line per path:
ms per batch of users, and whether the two agree.

    python tools/eval_bench.py [--batch 10000] [--reps 5] [--k 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA


@torch.no_grad()
def near_tie(U, I, bu, graph, top, k):
    """test_evaluate_matches_oracle's criterion on the device: every picked
    item is in the exact top-k of the float64 scores (train positives
    excluded) or within 1e-5 x max|score| of the exact k-th score."""
    s = U[bu].double() @ I.double().t()
    rp, col = graph.rowptr, graph.col
    users = bu.long()
    beg, end = rp[users], rp[users + 1]
    cnt = end - beg
    rows = torch.repeat_interleave(torch.arange(len(users), device=s.device), cnt)
    off = torch.arange(int(cnt.sum()), device=s.device) - \
        torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    items = col[torch.repeat_interleave(beg, cnt) + off].long() - graph.n_users
    s[rows, items] = -float("inf")
    kth = torch.topk(s, k, dim=1).values[:, k - 1]
    eps = 1e-5 * float(s[torch.isfinite(s)].abs().max())
    picked = torch.gather(s, 1, top[:, :k].long())
    exact = picked >= kth[:, None]
    ok = bool((picked >= kth[:, None] - eps).all())
    return {"check": "float64 near-tie (test_evaluate_matches_oracle)", "all_picks_ok": ok,
            "near_tie_users": int((~exact.all(dim=1)).sum()), "users": int(len(users)),
            "eps": eps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--dense", type=int, default=1, help="also time the GEMM + top-k path")
    ap.add_argument("--check64", type=int, default=1,
                    help="check every streamed pick against float64 scores (near-tie test)")
    a = ap.parse_args()
    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.evaluate import score_topk, topk_masked
    ds = SyntheticBipartite(a.users, a.items, a.edges, seed=0, test_frac=0)
    torch.manual_seed(0)
    m = LightGCN({"recdim": a.dim, "layer": 3, "lr": 1e-3, "decay": 1e-4, "device": "cuda:0",
                  "bpr_batch_size": 2048}, ds)
    U, I = m.eval_embeddings()
    bu = torch.randperm(a.users, device="cuda")[: a.batch]

    def stream():
        return score_topk(U[bu], I, bu, m.graph, a.k)

    def dense():
        return topk_masked((U[bu] @ I.t()).contiguous(), bu, m.graph, a.k)

    out = {}
    paths = (("stream", stream), ("dense", dense)) if a.dense else (("stream", stream),)
    for name, fn in paths:
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            r = fn()
        e.record()
        torch.cuda.synchronize()
        out[name] = r
        ms = s.elapsed_time(e) / a.reps
        flop = 2.0 * a.batch * a.items * a.dim
        print(json.dumps({"path": name, "batch_users": a.batch, "items": a.items, "dim": a.dim,
                          "k": a.k, "ms_per_batch": round(ms, 3),
                          "tflops_scores": round(flop / ms / 1e9, 1),
                          "frac_f32_mfma_peak": round(flop / ms / 1e9 / F32_PEAK_TFLOPS, 4),
                          "lib": os.path.basename(os.environ.get("MIREC_LIB", "libmirec.so")),
                          "rating_matrix_bytes": 0 if name == "stream" else 4 * a.batch * a.items}),
              flush=True)
    if a.check64:
        print(json.dumps(near_tie(U, I, bu, m.graph, out["stream"][1], a.k)), flush=True)
    if not a.dense:
        return
    si, di = out["stream"][1], out["dense"][1]
    same = torch.equal(si, di)
    rows_same = float((si == di).all(dim=1).float().mean())
    vdiff = float((out["stream"][0] - out["dense"][0]).abs().max())
    vmax = float(out["dense"][0].abs().max())
    # the two paths sum the d products in different orders: scores agree to
    # fp32 rounding, so near-tied items may swap places; the position-wise
    # scores of the two top-k lists agreeing within that rounding means
    # both are a top-k of the same ratings
    print(json.dumps({"agree_idx": same, "rows_identical_frac": round(rows_same, 6),
                      "max_val_diff": vdiff, "max_score": vmax,
                      "same_topk_values": vdiff <= 1e-6 * vmax}), flush=True)


if __name__ == "__main__":
    main()
