"""Ingest: the reference's Python line loop (restated in
oracle.parse_interaction_file, dataloader.py:93-126) vs the native
multi-threaded parser behind Loader, on a synthetic train file of C2 shape
(one line per user, ~20 items per line).  CPU only.  One JSON line.

    python tools/bench_ingest.py [--users 200000 --items-per-user 20 --threads 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=200_000)
    ap.add_argument("--items-per-user", type=int, default=20)
    ap.add_argument("--m-items", type=int, default=100_000)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    args = ap.parse_args()
    from furusato_recommend_amd.dataloader import parse_interactions
    from oracle.lightgcn_oracle import parse_interaction_file
    rng = np.random.default_rng(0)
    items = rng.integers(0, args.m_items, (args.users, args.items_per_user))
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "train.txt")
        with open(path, "w") as f:
            for u in range(args.users):
                f.write(str(u) + " " + " ".join(map(str, items[u])) + "\n")
        size = os.path.getsize(path)
        t0 = time.perf_counter()
        ref = parse_interaction_file(path)
        t_ref = time.perf_counter() - t0
        parse_interactions(path, n_threads=args.threads)  # warm page cache / pool
        t0 = time.perf_counter()
        uid, off, it, _, _ = parse_interactions(path, n_threads=args.threads)
        t_nat = time.perf_counter() - t0
        same = uid.tolist() == [u for u, _ in ref] and \
            it.tolist() == [x for _, row in ref for x in row]
    print(json.dumps({
        "metric": "ingest lines/s (train file, SURVEY §8 a1)",
        "lines": args.users, "items": int(it.size), "bytes": size,
        "reference_loop_s": round(t_ref, 3), "native_s": round(t_nat, 4),
        "reference_lines_per_s": round(args.users / t_ref, 1),
        "native_lines_per_s": round(args.users / t_nat, 1),
        "native_GB_per_s": round(size / t_nat / 1e9, 3), "threads": args.threads,
        "speedup": round(t_ref / t_nat, 1), "identical": bool(same)}))


if __name__ == "__main__":
    main()
