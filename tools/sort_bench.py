"""Time the key sorts of the training steps: mirec_key_sort_pairs (the
counting sort, csrc/keysort.hip) against torch.sort(stable=True) (the device
library's radix sort) on the shapes of C2 (BPR seeds: 6144 keys over 1.1 M
nodes), C4 (item-table gradient: 63 488 keys over 100 K items) and C3 (id-
table gradient: 1.76 M keys over 1.1 M rows), uniform and Zipf keys; every
result checked equal to the stable order.  One JSON line per case.

    python tools/sort_bench.py [--reps 50]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch

    from furusato_recommend_amd.rows import key_sort_pairs
    rng = np.random.default_rng(0)
    for name, n, nk in [("c2_seeds", 6144, 1_100_000), ("c4_tg", 63_488, 100_001),
                        ("c3_tg", 1_757_184, 1_100_001)]:
        for dist in ["uniform", "zipf"]:
            k = rng.integers(0, nk, n) if dist == "uniform" else np.minimum(rng.zipf(1.3, n) - 1, nk - 1)
            kt = torch.from_numpy(k.astype(np.int32)).cuda()
            ko, vo = key_sort_pairs(kt, nk)
            order = np.argsort(k, kind="stable")
            ok = bool(np.array_equal(vo.cpu().numpy(), order) and np.array_equal(ko.cpu().numpy(), k[order]))
            res = {}
            for impl in ["count", "torch"]:
                f = (lambda: key_sort_pairs(kt, nk)) if impl == "count" else (lambda: torch.sort(kt, stable=True))
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res[impl] = round(e0.elapsed_time(e1) / a.reps * 1e3, 1)
            print(json.dumps({"case": name, "keys": dist, "n": n, "nk": nk, "equal_stable_order": ok,
                              "count_us": res["count"], "torch_stable_sort_us": res["torch"],
                              "note": "count_us includes the workspace allocation of the wrapper"}),
                  flush=True)


if __name__ == "__main__":
    main()
