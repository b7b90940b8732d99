"""A/B timing of engine tuning switches on the C2 training step (1 GPU).

Prints, per variant, ms/step and the average time of every propagation
launch of the step in launch order (forward layers 1..L, backward layers
L-1..0), measured with HIP events on the launch stream.

  python tools/bench_variants.py [--steps 20] [--variants a,b,...]

An alternative build of libmirec.so is selected with MIREC_LIB=<path>.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "base": {},
    "no_hop_list": {"use_hop_list": False},
    "no_reuse": {"reuse_prescaled": False},
    "mask_only": {"use_hop_list": False, "reuse_prescaled": False},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2048)
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
    step_no = [0]

    def step():
        sample_triples(model.graph, B, 0, step_no[0] * B, u, p, n, err)
        step_no[0] += 1
        eng.train_step(emb, model.optim, u, p, n, 1e-4)

    for name in args.variants.split(","):
        for k, v in VARIANTS[name].items():
            setattr(eng, k, v)
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
        print(json.dumps({"variant": name, "ms_per_step": round(dt * 1e3, 4),
                          "launch_ms": launches, "prop_sum_ms": round(sum(launches), 4)}))
        for k in VARIANTS[name]:
            setattr(eng, k, {"use_hop_list": True, "reuse_prescaled": True}[k])


if __name__ == "__main__":
    main()
