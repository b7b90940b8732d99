"""Diagnostic: which rows make the full propagation launch slow on the Zipf
C2 variant (row subsets as row lists, natural vs shuffled order)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e), 3)


def main():
    from furusato_recommend_amd import Graph, SyntheticBipartite
    from furusato_recommend_amd._lib import IN_PRESCALED
    from furusato_recommend_amd.engine import PropagationEngine
    ds = SyntheticBipartite(1_000_000, 100_000, 20_000_000, seed=0, kind="zipf")
    g = Graph.from_interactions(ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, "cuda:0")
    eng = PropagationEngine(g, 64, 3, max_batch=2048, prune=True)
    N, nu = g.n_nodes, ds.n_users
    x = torch.randn(N, 64, device="cuda")
    y = torch.empty_like(x)
    allmask = torch.ones((N + 3) // 4, dtype=torch.int32, device="cuda") * 0x01010101
    dev = "cuda"
    deg = torch.from_numpy(g.degree()).to(dev)
    item_ids = torch.arange(nu, N, device=dev)
    dg = deg[nu:]
    sets0 = {
        "no rows (segments only)": torch.zeros(1, dtype=torch.int32, device=dev)[:0],
        "items 64<deg<=2048": item_ids[(dg > 64) & (dg <= 2048)].int(),
        "items deg<=64": item_ids[dg <= 64].int(),
        "items deg>2048 (skipped rows)": item_ids[dg > 2048].int(),
    }
    for name, rows in sets0.items():
        cnt = torch.tensor([rows.numel()], dtype=torch.int32, device=dev)
        r = rows if rows.numel() else torch.zeros(1, dtype=torch.int32, device=dev)
        t = timed(lambda: eng._prop(in_mode=IN_PRESCALED, x_in=x, out=y, row_mask=allmask,
                                    row_list=r, row_count=cnt, row_list_cap=max(rows.numel(), 1)))
        print(name, rows.numel(), "ms", t, flush=True)
    sets = {
        "users natural": torch.arange(nu, dtype=torch.int32, device=dev),
        "users shuffled": torch.randperm(nu, device=dev).int(),
        "items natural": torch.arange(nu, N, dtype=torch.int32, device=dev),
        "items shuffled": (nu + torch.randperm(N - nu, device=dev)).int(),
        "first 100k users": torch.arange(100_000, dtype=torch.int32, device=dev),
    }
    for name, rows in sets.items():
        cnt = torch.tensor([rows.numel()], dtype=torch.int32, device=dev)
        t = timed(lambda: eng._prop(in_mode=IN_PRESCALED, x_in=x, out=y, row_mask=allmask,
                                    row_list=rows, row_count=cnt, row_list_cap=rows.numel()))
        print(name, rows.numel(), "ms", t, flush=True)
    print("full", timed(lambda: eng._prop(in_mode=IN_PRESCALED, x_in=x, out=y)), flush=True)


if __name__ == "__main__":
    main()
