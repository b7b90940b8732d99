"""Recall@20 after E epochs on a graph with structure (SyntheticBipartite
kind='cluster'): the HIP engine and the CPU oracle trained on the same
UniformSample triples (numpy seeds 100+e), evaluated with trainer.py /
metric.py semantics.  One JSON line per epoch.

    python tools/quality.py [--epochs 5 --users 4000 --items 800 --edges 80000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--users", type=int, default=4000)
    ap.add_argument("--items", type=int, default=800)
    ap.add_argument("--edges", type=int, default=80_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--lr", type=float, default=5e-3)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--no-oracle", action="store_true")
    args = ap.parse_args()
    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.evaluate import evaluate
    from oracle.lightgcn_oracle import OracleLightGCN, uniform_sample
    from oracle.lightgcn_oracle import evaluate as oracle_evaluate
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=3, kind="cluster",
                            test_frac=0.2)
    torch.manual_seed(0)
    m = LightGCN({"recdim": args.dim, "layer": args.layers, "lr": args.lr, "decay": 1e-4,
                  "device": "cuda:0", "bpr_batch_size": args.batch}, ds)
    o = None if args.no_oracle else OracleLightGCN(
        ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, args.dim, args.layers, args.lr, 1e-4,
        emb=m.all_embedding.weight.detach().cpu().clone())
    for e in range(args.epochs):
        np.random.seed(100 + e)
        S = uniform_sample(ds.n_users, ds.m_items, ds.allPos, ds.trainDataSize)
        t0 = time.perf_counter()
        lg = float(m.OneEpoch(S[:, 0], S[:, 1], S[:, 2]))
        t_gpu = time.perf_counter() - t0
        r = evaluate(m, ds.testDict, (20,), batch=2000)
        line = {"epoch": e + 1, "loss": round(lg, 6), "recall@20": round(float(r["recall"][0]), 5),
                "ndcg@20": round(float(r["ndcg"][0]), 5), "epoch_s_gpu": round(t_gpu, 3)}
        if o is not None:
            t0 = time.perf_counter()
            lo = o.OneEpoch(S[:, 0], S[:, 1], S[:, 2], args.batch)
            line["epoch_s_cpu_oracle"] = round(time.perf_counter() - t0, 3)
            out = o.propagated()
            ro = oracle_evaluate(out[:ds.n_users], out[ds.n_users:], ds.testDict, ds.allPos, (20,))
            line.update(oracle_loss=round(lo, 6), oracle_recall20=round(float(ro["recall"][0]), 5))
            w = m.all_embedding.weight.detach().cpu().double()
            line["table_rel_diff"] = float((w - o.emb.detach().double()).abs().max()
                                           / o.emb.detach().double().abs().max())
        line["chance_recall20"] = round(20 / ds.m_items, 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
