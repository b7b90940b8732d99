"""Per-rank compute of the sparse-seed data-parallel step at world size W,
simulated on ONE GPU (the scaling rehearsal; 8-GPU runs are the driver's).

Rank 0's step at world W: sample its user shard, pruned forward, BPR with
grad_scale 1/W, pack seeds, (all-gather), merge the W ranks' seeds, frontier
of the union, pruned backward with fused Adam.  The other W-1 ranks' packed
seeds are produced once up front by running their own shards' forward + BPR;
each timed step concatenates them behind rank 0's fresh seeds (a device
copy standing in for the all-gather's output write).  What is NOT measured:
the RCCL all-gather itself (W x 3B x (4 + 8D) bytes, 3.2 MB per rank at C2).

  python tools/bench_world_sim.py [--worlds 1,2,4,8] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--sparse-filters", default="auto",
                    help="comma list of engine.sparse_filter values to compare")
    ap.add_argument("--modes", default="sparse",
                    help="comma list of DataParallel modes: sparse (replicated last "
                         "layer + Adam) and/or sharded (rank 0's row shard only, plus the "
                         "local copies and re-prescale of the all-gather; the RCCL "
                         "transfer itself is not measured)")
    args = ap.parse_args()
    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.engine import sample_triples
    dev = torch.device("cuda:0")
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0)
    torch.manual_seed(0)
    cfg = {"recdim": args.dim, "layer": 3, "lr": 1e-3, "decay": 1e-4, "device": "cuda:0",
           "bpr_batch_size": args.batch}
    model = LightGCN(cfg, ds)
    eng = model.engine
    emb = model.all_embedding.weight.data
    B = args.batch
    u = torch.empty(B, dtype=torch.int32, device=dev)
    p, n = torch.empty_like(u), torch.empty_like(u)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    configs = [(int(w), f, m) for w in args.worlds.split(",")
               for f in args.sparse_filters.split(",") for m in args.modes.split(",")]
    for W, filt, mode in configs:
        eng.sparse_filter = filt
        last_rows, stage = None, None
        if mode == "sharded":
            N = model.graph.n_nodes
            S = (N + W - 1) // W
            bm = torch.zeros((N + 15) // 16 * 4, dtype=torch.int32, device=dev)
            bm.view(torch.uint8)[0:N:W] = 1  # rank 0's interleaved shard (dist.py)
            last_rows = eng.static_row_lists(bm)
            stage = torch.empty(W, S, args.dim, device=dev)
        others = []
        for r in range(1, W):
            sample_triples(model.graph, B, 0, 10**9, u, p, n, err, r, W)
            out = eng.forward_for_batch(emb, u, p, n)
            eng.bpr(out, emb, u, p, n, 1e-4, grad_scale=1.0 / W)
            k, sp, se = eng.export_seeds()
            others.append((k.clone(), sp.clone(), se.clone()))
        eng.invalidate_prescaled()
        step_no = [0]

        def step():
            sample_triples(model.graph, B, 0, step_no[0] * B, u, p, n, err, 0, W)
            step_no[0] += 1
            out = eng.forward_for_batch(emb, u, p, n)
            eng.bpr(out, emb, u, p, n, 1e-4, grad_scale=1.0 / W)
            k, sp, se = eng.export_seeds()
            keys = torch.cat([k] + [o[0] for o in others])
            rp = torch.cat([sp] + [o[1] for o in others])
            re = torch.cat([se] + [o[2] for o in others])
            eng.import_seeds(keys, rp, re)
            eng.backward(emb, adam=model.optim, last_rows=last_rows)
            if mode == "sharded":  # the all-gather's local copies + re-prescale
                N = emb.shape[0]
                stage[0, : len(range(0, N, W))].copy_(emb[0:N:W])
                full = N // W
                emb[: full * W].view(full, W, -1).copy_(stage[:, :full].transpose(0, 1))
                eng.invalidate_prescaled()

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        eng.prop_events = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        ev, eng.prop_events = eng.prop_events, None
        per = len(ev) // args.steps
        launches = []
        for j in range(per):
            ms = [ev[s * per + j][0].elapsed_time(ev[s * per + j][1]) for s in range(args.steps)]
            launches.append(round(sum(ms) / len(ms), 4))
        f1 = int((eng.bm_hop.view(torch.uint8)[: model.graph.n_nodes] != 0).sum())
        print(json.dumps({"world": W, "mode": mode, "sparse_filter": filt,
                          "ms_per_step_rank": round(dt * 1e3, 4),
                          "edges_per_s_projected": round(W * B / dt, 1),
                          "launch_ms": launches, "union_F1_rows": f1}), flush=True)


if __name__ == "__main__":
    main()
