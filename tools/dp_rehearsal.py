"""Multi-rank rehearsal of the data-parallel LightGCN step on ONE GPU.

Every rank runs on cuda:0 and the collectives go through gloo (RCCL needs
one GPU per rank); everything else is bench.py's N-rank path: user-sharded
on-device sampling, sparse-seed all-gather + merge (or the dense
all-reduce), pruned backward with fused Adam.  Checks that the replicas stay
bit-identical and that the 2-rank step equals one process stepping on the
union of the ranks' batches.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29531 tools/dp_rehearsal.py [--model lgn|sage|sasrec]
        [--mode sparse|dense]
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def autograd_models(args, rank, world, dev):
    """GraphSAGE / SASRec under DenseGradDataParallel: different inits are
    fixed by the broadcast, every rank steps on its own user shard, and the
    gradient all-reduce keeps the replicas bit-identical."""
    import numpy as np

    from furusato_recommend_amd import GraphSAGE, SASRec, SyntheticBipartite
    from furusato_recommend_amd.dist import DenseGradDataParallel
    ds = SyntheticBipartite(50_000, 5_000, 500_000, seed=0)
    torch.manual_seed(100 + rank)
    cfg = {"recdim": 64, "layer": 2, "lr": 1e-3, "decay": 1e-4, "device": "cuda:0",
           "bpr_batch_size": 512, "heads": 2, "fanouts": [10, 5]}
    m = GraphSAGE(cfg, ds) if args.model == "sage" else SASRec(cfg, ds)
    dp = DenseGradDataParallel(m)
    rng = np.random.default_rng(rank)
    losses = []
    for i in range(args.steps):
        if args.model == "sage":
            u, p, n = m.sample(512, seed=5, offset=i * 512, shard=rank, n_shards=world)
        else:
            u = rng.integers(0, ds.n_users, 512) // world * world + rank
            u = np.minimum(u, ds.n_users - 1)
            p = torch.randint(0, ds.m_items, (512,), device=dev)
            n = torch.randint(0, ds.m_items, (512,), device=dev)
        losses.append(float(dp.step(u, p, n)))
    torch.cuda.synchronize()
    flat = torch.cat([q.detach().reshape(-1).cpu() for q in m.parameters()])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        same = all(torch.equal(gathered[0], g) for g in gathered[1:])
        ok = same and all(np.isfinite(losses))
        print(json.dumps({"world": world, "model": args.model, "replicas_identical": same,
                          "losses": [round(x, 5) for x in losses], "ok": bool(ok)}), flush=True)
        if not ok:
            sys.exit(1)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lgn", choices=["lgn", "sage", "sasrec"])
    ap.add_argument("--mode", default="sparse")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--users", type=int, default=200_000)
    ap.add_argument("--items", type=int, default=20_000)
    ap.add_argument("--edges", type=int, default=4_000_000)
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    if args.model != "lgn":
        return autograd_models(args, rank, world, dev)
    from furusato_recommend_amd import LightGCN, SyntheticBipartite
    from furusato_recommend_amd.dist import DataParallel
    from furusato_recommend_amd.engine import sample_triples
    ds = SyntheticBipartite(args.users, args.items, args.edges, seed=0)
    cfg = {"recdim": 64, "layer": 3, "lr": 1e-3, "decay": 1e-4, "device": "cuda:0",
           "bpr_batch_size": args.batch}
    torch.manual_seed(100 + rank)  # different inits: the broadcast must fix them
    model = LightGCN(cfg, ds)
    emb = model.all_embedding.weight.data
    dp = DataParallel(model.engine, emb, model.optim, mode=args.mode)
    B = args.batch
    batches = []
    for i in range(args.steps):
        u = torch.empty(B, dtype=torch.int32, device=dev)
        p, n = torch.empty_like(u), torch.empty_like(u)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        sample_triples(model.graph, B, 11, i * B, u, p, n, err, rank, world)
        dp.step(u, p, n, cfg["decay"])
        batches.append(torch.stack([u, p, n]).cpu())
    torch.cuda.synchronize()
    table = emb.detach().cpu()
    gathered = [torch.empty_like(table) for _ in range(world)]
    dist.all_gather(gathered, table)
    all_batches = [None] * world
    dist.all_gather_object(all_batches, batches)
    if rank == 0:
        same = all(torch.equal(gathered[0], g) for g in gathered[1:])
        # one process on the union batches (rank-major order), same init
        torch.manual_seed(100)
        ref = LightGCN(dict(cfg, bpr_batch_size=B * world), ds)
        for i in range(args.steps):
            uni = torch.cat([all_batches[r][i] for r in range(world)], dim=1).to(dev)
            ref.engine.train_step(ref.all_embedding.weight.data, ref.optim,
                                  uni[0].contiguous(), uni[1].contiguous(),
                                  uni[2].contiguous(), cfg["decay"])
        torch.cuda.synchronize()
        r = ref.all_embedding.weight.detach().cpu().double()
        err = float((gathered[0].double() - r).abs().max() / r.abs().max())
        print(json.dumps({"world": world, "mode": args.mode, "replicas_identical": same,
                          "rel_err_vs_union_batch": err, "ok": bool(same and err < 1e-5)}),
              flush=True)
        if not (same and err < 1e-5):
            sys.exit(1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
