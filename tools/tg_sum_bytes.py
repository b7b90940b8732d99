"""Algorithmic bytes of the C3 sorted table-gradient sum (tg_sum_kernel) per
launch, from the row groups one real C3 step hands to TableGrad.accumulate,
and — with a rocprofv3 FETCH_SIZE / WRITE_SIZE pass directory — the counter
bytes of the same kernel beside them.

    python tools/tg_sum_bytes.py                     # counts, one JSON line
    python tools/tg_sum_bytes.py --fetch DIR --write DIR [--out FILE]

Algorithmic (every operand once): the sort's keys and values read (8 B per
entry), one weight per target (4 B), every gradient row read ONCE (inner
entries' rows; a leaf group's g_out row per target), the summed rows written
once per distinct row id (d x 4 B) and its stamp (4 B).  The pull form reads
a target's g_out row once per child entry instead ("pull_read_bytes")."""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counts(B=2048, fan=(25, 10), dim=128):
    import torch

    from furusato_recommend_amd import GraphSAGE, SyntheticBipartite
    from furusato_recommend_amd import graphsage as G
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0)
    torch.manual_seed(2020)
    m = GraphSAGE({"recdim": dim, "layer": len(fan), "fanouts": list(fan), "lr": 1e-3,
                   "decay": 1e-7, "device": "cuda:0", "bpr_batch_size": B}, ds)
    seen = []
    orig = G.TableGrad.accumulate

    def spy(self, groups):
        seen.append([(ids.clone(), int(g.shape[0]), int(k)) for ids, g, k, *_ in groups])
        return orig(self, groups)
    G.TableGrad.accumulate = spy
    u, p, n = m.sample(B, seed=7, offset=0)
    m.stageOne(u, p, n)
    torch.cuda.synchronize()
    G.TableGrad.accumulate = orig
    groups = seen[-1]
    n_ent = sum(ids.numel() for ids, _, _ in groups)
    valid = torch.cat([ids[ids >= 0] for ids, _, _ in groups])
    n_tgt = sum(nt for _, nt, _ in groups)
    rows_once = 0
    for ids, nt, k in groups:
        if k == 1:
            rows_once += int((ids >= 0).sum())
        else:  # targets with at least one valid child
            rows_once += int(((ids.view(nt, k) >= 0).any(1)).sum())
    distinct = int(torch.unique(valid).numel())
    reuse = reuse_windows(groups)
    rb = dim * 4
    alg = 8 * n_ent + 4 * n_tgt + rb * rows_once + (rb + 4) * distinct
    return {"entries": n_ent, "valid_entries": int(valid.numel()), "targets": n_tgt,
            "grad_rows_once": rows_once, "distinct_rows": distinct,
            "groups": [(int(ids.numel()), nt, k) for ids, nt, k in groups],
            "algorithmic_bytes": alg,
            "pull_read_bytes": 8 * n_ent + 4 * n_tgt + rb * int(valid.numel()),
            "write_bytes": (rb + 4) * distinct, "reuse": reuse}


def reuse_windows(groups, windows=(8, 64, 512, 4096, 32768)):
    """How much of the pull form's gradient-row re-reading a window of sorted
    entries could absorb: the entries in sort order (row id, entry order),
    each tagged with the gradient row it reads (its target's g_out row for a
    fanout group, its own row for a k = 1 group); per window of W consecutive
    sorted entries, the distinct gradient rows it reads.  distinct / entries
    = the fraction of row reads a perfect W-entry reuse (LDS or cache) would
    still issue; 1.0 = no reuse at that scale.  The VERDICT r5 variant (a
    fanout group's entries ordered by (row, target)) changes only the order
    inside a run of equal row ids, i.e. windows of one run."""
    import torch
    keys, src, base = [], [], 0
    for ids, nt, k in groups:
        ids = ids.view(-1)
        e = torch.arange(ids.numel(), device=ids.device)
        tgt = (e // k + base) if k > 1 else (e + base)
        base += nt if k > 1 else ids.numel()
        ok = ids >= 0
        keys.append(ids[ok].long())
        src.append(tgt[ok])
    keys, src = torch.cat(keys), torch.cat(src)
    order = torch.sort(keys, stable=True).indices
    s = src[order]
    k_sorted = keys[order]
    runs = int(torch.unique_consecutive(k_sorted).numel())
    out = {"valid_entries": int(s.numel()), "runs": runs,
           "mean_run": round(s.numel() / max(runs, 1), 3)}
    for W in windows:
        m = s.numel() // W * W
        blk = torch.sort(s[:m].view(-1, W), dim=1).values
        d = int((blk[:, 1:] != blk[:, :-1]).sum()) + blk.shape[0]
        out[f"distinct_per_entry_W{W}"] = round(d / max(m, 1), 4)
    return out


def pmc(dirname, counter, kernel="tg_sum_kernel"):
    vals = []
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--counts")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.fetch:
        c = json.load(open(a.counts))
        fs, ws = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
        rd = 2 * 1024 * sum(fs) / max(len(fs), 1)  # gfx950: 2 x FETCH_SIZE x 1 KiB
        wr = 1024 * sum(ws) / max(len(ws), 1)
        res = dict(c, kernel="tg_sum_kernel (C3 sorted table-gradient sum, pass 1)",
                   launches=[len(fs), len(ws)], read_bytes=rd, write_bytes_counter=wr,
                   hbm_bytes_per_launch=rd + wr,
                   counter_over_algorithmic=round((rd + wr) / c["algorithmic_bytes"], 3),
                   correction="read = 2*FETCH_SIZE*1024 (gfx950), write = WRITE_SIZE*1024; "
                              "FETCH_SIZE counts L2 misses, Infinity-Cache hits included")
        s = json.dumps(res, indent=1)
        if a.out:
            open(a.out, "w").write(s + "\n")
        print(s)
    else:
        print(json.dumps(counts()), flush=True)
