"""Config C4 (BASELINE.json configs[3]): SASRec L=2 heads=2 d=128 maxlen=50,
1M users with synthetic sequences of length U[5, 50] over 100K items, one
MI355X.  A step is one stageOne (model/sasrec.py:437-474 per batch): B
sequences through two attention blocks + pooling, the item tower on the
positive and negative items, BPR + norm loss, backward, Adam.  Prints one
JSON line: positive-edges/s and the attention kernels' roofline (live HIP
events on their launch stream).

Training runs on packed sequences (only the real positions; padding never
reaches them under the causal mask).  Algorithmic work of one attention
launch over B sequences of lengths T_b x h heads (dense T_b x T_b scores):
  forward : 4 T_b^2 dh FLOP per (sequence, head); reads qkv (T_b 3d 4 B),
            writes out (T_b d 4 B)
  backward: 10 T_b^2 dh FLOP (S recomputed, dV, dP, dQ, dK); reads qkv and
            dO, writes dqkv
The bound is whichever of HBM (8 TB/s) and f32 MFMA (157.3 TFLOP/s,
MI355X_MICROARCH.md) takes longer for that work.

    python tools/bench_sasrec.py [--steps K --warmup W]
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

HBM_PEAK = 8.0e12
F32_MFMA_PEAK = 157.3e12


class _DS:
    def __init__(self, n_users, m_items):
        self.n_users, self.m_items = n_users, m_items


def cpu_baseline(m, seq, B, heads, rng):
    """The oracle's restatement of sasrec.py:385-435 (torch CPU fp32, padded
    batch as the reference's pad_sequence, dropout off) on one batch of the
    same workload: blocks + pool, item tower, BPR + embedding-norm loss,
    backward, torch Adam over every parameter."""
    import torch.nn.functional as F

    from oracle import lightgcn_oracle as O
    L = m.num_layers
    cpu = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    p = {}
    for i in range(L):
        a = f"attn_layers.{i}."
        p.update({f"ln1_w{i}": cpu[f"attn_norm_layers.{i}.weight"],
                  f"ln1_b{i}": cpu[f"attn_norm_layers.{i}.bias"],
                  f"in_w{i}": cpu[a + "in_proj_weight"], f"in_b{i}": cpu[a + "in_proj_bias"],
                  f"out_w{i}": cpu[a + "out_proj.weight"], f"out_b{i}": cpu[a + "out_proj.bias"],
                  f"ln2_w{i}": cpu[f"ffn_norm_layers.{i}.weight"],
                  f"ln2_b{i}": cpu[f"ffn_norm_layers.{i}.bias"],
                  f"ffn_w{i}": cpu[f"ffn_layers.{i}.weight"], f"ffn_b{i}": cpu[f"ffn_layers.{i}.bias"]})
    opt = torch.optim.Adam(list(cpu.values()), lr=1e-3)
    W = cpu["item_id_embedding.weight"]

    def tower(x):
        for j in range(L - 1):
            x = F.linear(x, cpu[f"item_linears.{j}.weight"], cpu[f"item_linears.{j}.bias"]).relu()
        return F.linear(x, cpu["item_last_proj.weight"], cpu["item_last_proj.bias"])

    import bench
    threads = bench.host_threads()
    torch.set_num_threads(threads)
    T = seq.max_len
    k = 3
    times = []
    for i in range(k + 1):  # 1 warm-up step, then the mean of k
        u = torch.from_numpy(rng.integers(0, seq.items.shape[0], B))
        items = seq.items.cpu()[u].long()
        length = seq.length.cpu()[u]
        pos = items[torch.arange(B), (torch.rand(B) * length).long()]
        neg = torch.randint(0, m.m_item, (B,))
        t0 = time.perf_counter()
        opt.zero_grad()
        mask = (torch.arange(T)[None, :] < length[:, None]).float().unsqueeze(2)
        ue = O.sasrec_forward_user(W[items.clamp(min=0)] * mask, length, p, heads, L)
        pe, ne = tower(W[pos]), tower(W[neg])
        loss = F.softplus((ue * ne).sum(1) - (ue * pe).sum(1)).mean() + 1e-4 * W.norm(2) / B
        loss.backward()
        opt.step()
        if i:
            times.append(time.perf_counter() - t0)
    t = sum(times) / k
    return {"value": round(B / t, 2), "unit": "positive-edges/s", "cores": threads,
            "threads": threads, "os_cpu_count": os.cpu_count(), "kind": "port",
            "cpu": bench.cpu_model(), "warmup": 1, "k": k, "step_s": round(t, 3),
            "step_s_each": [round(x, 3) for x in times],
            "sample": f"1 warm-up + mean of {k} training steps (B={B}, padded T={T}) of the C4 "
                      f"workload, a fresh batch each"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--maxlen", type=int, default=50)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--blas", default="", choices=["", "cublas", "cublaslt"],
                    help="BLAS backend of the projections (cublas = rocBLAS, cublaslt = "
                         "hipBLASLt on ROCm; default: the model's choice per step mode)")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: replay the captured HIP graph of the step; 0: eager step")
    ap.add_argument("--attn-buckets", type=int, default=0,
                    help="0: every packed sequence on the 64-row attention kernel (A/B)")
    ap.add_argument("--attn-impl", default="hybrid", choices=["hybrid", "wave", "block"],
                    help="attention core (sasrec.ATTN_IMPL): wave forward + workgroup "
                         "backward (default), one wave, or one workgroup per (sequence, head)")
    ap.add_argument("--table-grad", default="sorted", choices=["sorted", "atomic", "dense"],
                    help="item table gradient: sorted (deterministic) / atomic S + fused "
                         "table Adam, or the materialised gradient + dense Adam")
    ap.add_argument("--fused-rows", type=int, default=1,
                    help="0: the torch composition of dropout / residual / LayerNorm (A/B)")
    ap.add_argument("--rehearse", action="store_true",
                    help="under torch.distributed.run: every rank on cuda:0, gloo collectives "
                         "(the data-parallel path on one GPU; not a throughput measurement)")
    ap.add_argument("--table-exchange", default="auto", choices=["auto", "routed", "dense"])
    args = ap.parse_args()
    from furusato_recommend_amd import SASRec, sasrec as S
    from furusato_recommend_amd.sasrec import SequenceData
    S.ATTN_IMPL = args.attn_impl
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    gpu = 0 if args.rehearse else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        import torch.distributed as dist

        from furusato_recommend_amd.dist import DenseGradDataParallel, init_distributed
        init_distributed("gloo" if args.rehearse else "nccl", dev)
    torch.manual_seed(2020)
    seq = SequenceData.synthetic(args.users, args.items, dev, max_len=args.maxlen, min_len=5,
                                 seed=0)
    m = SASRec({"recdim": args.dim, "layer": args.layers, "heads": args.heads, "lr": 1e-3,
                "decay": 1e-4, "device": "cuda:0", "bpr_batch_size": args.batch,
                "dropout_p": 0.2, **({"blas": args.blas} if args.blas else {}),
                "fused_rows": bool(args.fused_rows), "attn_buckets": bool(args.attn_buckets),
                "graph": bool(args.graph), "table_grad": args.table_grad},
               _DS(args.users, args.items),
               sequences=seq)
    dp = None
    if world > 1:
        dp = DenseGradDataParallel(m, table_exchange=None if args.table_exchange == "auto"
                                   else args.table_exchange)
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(7)

    rng = np.random.default_rng(7)
    step = [0]

    def batch():
        # users uniform, drawn on the host like the reference's UniformSample
        # (so the packed batch is sized without a device sync); positive = a
        # random element of the user's sequence; negative uniform (timing
        # workload: no rejection of positives)
        u_h = rng.integers(0, args.users // world, B) * world + rank  # the rank's user shard
        u = m._upload(u_h)  # pinned staging: no stream sync
        step[0] += 1
        pn = m.sample_pairs(u, 7, step[0] * B)  # one launch: [pos ; neg]
        return u_h, pn[0], pn[1]

    run = m.stageOne if dp is None else dp.step
    for _ in range(args.warmup):
        run(*batch())
    torch.cuda.synchronize()
    if dp is not None:
        dp.comm_events = []
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run(*batch())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    comm = None
    if dp is not None:
        from furusato_recommend_amd.dist import _elapsed_ms
        cm = _elapsed_ms(dp.comm_events) / args.steps
        dp.comm_events = None
        t = torch.tensor([dt, cm], dtype=torch.float64, device="cpu" if args.rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, cm = float(t[0]), float(t[1])
        comm = {"backend": dist.get_backend(), "world_size": world,
                "table_exchange": dp.table_exchange, "comm_ms_per_step": round(cm, 4),
                "exchange_bytes_per_rank": dp.last_exchange_bytes,
                "step": "captured, split around the exchange" if m.config["graph"] else "eager"}
        if rank == 0:
            print(json.dumps({"metric": "SASRec BPR positive-edges/sec (C4), data parallel",
                              "value": round(world * args.steps * B / dt, 1),
                              "unit": "positive-edges/s", "ms_per_step_rank": round(1e3 * dt / args.steps, 3),
                              "rehearsal": bool(args.rehearse), "comm": comm}), flush=True)
        dist.destroy_process_group()
        return
    # per-launch attention timing: a few eager steps of the same kernels
    # (events on the launch stream; a replayed graph records none)
    graph_mode = m.config["graph"]
    m.config["graph"] = False
    S.ATTN_EVENTS = []
    S.ATTN_REPEAT = 20  # back-to-back launches: kernel time, no host gaps
    for _ in range(5):
        m.stageOne(*batch())
    torch.cuda.synchronize()
    ev, S.ATTN_EVENTS = S.ATTN_EVENTS, None
    S.ATTN_REPEAT = 1
    m.config["graph"] = graph_mode

    kinds = {}
    for kind, s, e, (b, T, h, dh), offs, reps in ev:
        d = h * dh
        if offs is not None:  # packed: sum over the real sequence lengths
            lens = np.diff(offs.cpu().numpy().astype(np.int64))
            t2, t1 = float((lens * lens).sum()), float(lens.sum())
        else:
            t2, t1 = float(b) * T * T, float(b) * T
        if kind == "fwd":
            fl = 4.0 * t2 * dh * h
            by = 4.0 * t1 * (3 * d + d)
        else:
            fl = 10.0 * t2 * dh * h
            by = 4.0 * t1 * (3 * d + d + 3 * d)
        k = kinds.setdefault(kind, [0, 0.0, 0.0, 0.0])
        k[0] += 1
        k[1] += s.elapsed_time(e) / reps
        k[2] += fl
        k[3] += by
    roof = {}
    for kind, (cnt, ms, fl, by) in kinds.items():
        t = ms / cnt * 1e-3
        fl, by = fl / cnt, by / cnt  # per launch
        t_hbm, t_mfma = by / HBM_PEAK, fl / F32_MFMA_PEAK
        if t_hbm >= t_mfma:
            roof[kind] = {"bound": "hbm", "achieved": round(by / t / 1e9, 1), "peak": 8000.0,
                          "unit": "GB/s", "frac": round(t_hbm / t, 4)}
        else:
            roof[kind] = {"bound": "mfma", "achieved": round(fl / t / 1e12, 2), "peak": 157.3,
                          "unit": "TFLOP/s", "frac": round(t_mfma / t, 4)}
        roof[kind].update(avg_launch_ms=round(ms / cnt, 4), launches_per_step=cnt / 5,
                          flop_per_launch=fl, bytes_per_launch=by,
                          timing="HIP events around 20 back-to-back launches on one "
                                 "step's operands (kernel time, no host gaps), / 20")
    cpu = cpu_baseline(m, seq, B, args.heads, rng) if args.cpu_baseline else None
    print(json.dumps({
        "metric": "SASRec BPR positive-edges/sec (C4)",
        "value": round(args.steps * B / dt, 1), "unit": "positive-edges/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
        "dtype": "f32", "data": "synthetic sequences U[5,%d], random-init weights" % args.maxlen,
            "gemm_arith": "f32 products as an exact three-term bf16 split on bf16 MFMA (f32-class error: DESIGN.md section 4, profiles/round3c_gemm_split_accuracy.jsonl)",
        "config": {"workload": "C4: SASRec L=%d heads=%d d=%d maxlen=%d, %d users x %d items"
                   % (args.layers, args.heads, args.dim, args.maxlen, args.users, args.items),
                   "bpr_batch": B, "step": "HIP graph replay" if graph_mode else "eager"},
        "attention_roofline": roof, "cpu_baseline": cpu}), flush=True)


if __name__ == "__main__":
    main()
