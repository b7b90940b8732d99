"""Time the C3 sorted table-gradient sum (TableGrad.accumulate: prep, radix
sort, tg_sum, block sums, fixup) on the row groups of one real C3 step, and
checksum its result, for A/B builds of csrc/tablegrad.hip (select the
library with MIREC_LIB).  One JSON line: ms per accumulate (HIP events over
REPS back-to-back calls), the stamped row count and a float64 sum / bit hash
of the stamped rows (equal hashes = bitwise equal sums).

    python tools/tg_bench.py [--reps 50]"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    import torch

    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    from furusato_recommend_amd import graphsage as G
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    torch.manual_seed(2020)
    m = GraphSAGE({"recdim": 128, "layer": 2, "fanouts": [25, 10], "lr": 1e-3, "decay": 1e-7,
                   "device": "cuda:0", "bpr_batch_size": a.batch}, ds)
    seen = []
    orig = G.TableGrad.accumulate

    def spy(self, groups):
        seen.append((self, [tuple(x.clone() if torch.is_tensor(x) else x for x in g) for g in groups]))
        return orig(self, groups)
    G.TableGrad.accumulate = spy
    u, p, n = m.sample(a.batch, seed=7, offset=0)
    m.stageOne(u, p, n)
    torch.cuda.synchronize()
    G.TableGrad.accumulate = orig
    tg, groups = seen[-1]
    for _ in range(3):
        tg.accumulate(groups)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        tg.accumulate(groups)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    rows = (tg.stamp == tg.gen).nonzero().squeeze(1)
    s = tg.acc[rows].contiguous()
    h = hashlib.sha1(s.cpu().numpy().tobytes() + rows.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(os.environ.get("MIREC_LIB", "libmirec.so")),
                      "ms_per_accumulate": round(ms, 4), "reps": a.reps,
                      "entries": sum(int(g[0].numel()) for g in groups),
                      "stamped_rows": int(rows.numel()), "sum_f64": float(s.double().sum()),
                      "abs_f64": float(s.double().abs().sum()), "hash": h}), flush=True)


if __name__ == "__main__":
    main()
