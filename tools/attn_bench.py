"""Device time of the SASRec attention kernels (csrc/attn_wave.hip: one wave
per (sequence, head); csrc/attention.hip: one workgroup per (sequence,
head)) on packed sequences, for several batch sizes and length mixes — does
a launch scale with its work (throughput-bound) or stay flat (latency)?
One JSON line per (impl, mix, batch).

    python tools/attn_bench.py [--reps 20] [--heads 2] [--dh 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--dh", type=int, default=64)
    ap.add_argument("--batches", default="512,2048,8192")
    ap.add_argument("--mixes", default="c4,16,32,64")
    ap.add_argument("--order", type=int, default=1, help="wave kernels: longest sequences first")
    a = ap.parse_args()
    from furusato_recommend_amd import _lib
    lib, st, chk = _lib.lib, _lib.stream_handle(), _lib.check
    H, dh = a.heads, a.dh
    d = H * dh
    g = torch.Generator().manual_seed(0)
    for mix in a.mixes.split(","):
        for B in (int(x) for x in a.batches.split(",")):
            if mix == "c4":
                lens = torch.randint(5, 51, (B,), generator=g)
            else:
                lens = torch.full((B,), int(mix))
            offs = torch.zeros(B + 1, dtype=torch.int32)
            offs[1:] = torch.cumsum(lens, 0)
            offs = offs.cuda()
            n = int(lens.sum())
            qkv = torch.randn(n, 3 * d, device="cuda")
            out = torch.empty(n, d, device="cuda")
            lse = torch.empty(n, H, device="cuda")
            dout = torch.randn(n, d, device="cuda")
            dqkv = torch.empty_like(qkv)
            delta = torch.empty_like(lse)
            bp = -(-B // 4) * 4  # packs start 16-byte aligned
            order = torch.empty(bp + 4 + 8 * B, dtype=torch.int32, device="cuda")
            chk(lib.mirec_attention_length_order(offs.data_ptr(), B, order.data_ptr(),
                                                 order[bp:].data_ptr(), None, 0, 0, st), "ord")
            op = order.data_ptr() if a.order else None
            t2 = float((lens.double() ** 2).sum())
            by_f = 4.0 * n * 4 * d
            by_b = 4.0 * n * 7 * d
            runs = {
                "wave_fwd": lambda: chk(lib.mirec_attention_wave_fwd(
                    qkv.data_ptr(), offs.data_ptr(), op, B, 0, H, dh, out.data_ptr(), lse.data_ptr(),
                    0, st), "wave_fwd"),
                "wave_bwd": lambda: chk(lib.mirec_attention_wave_bwd(
                    qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), dout.data_ptr(),
                    offs.data_ptr(), op, B, 0, H, dh, dqkv.data_ptr(), delta.data_ptr(), st),
                    "wave_bwd"),
                "block_fwd": lambda: chk(lib.mirec_attention_varlen_fwd(
                    qkv.data_ptr(), offs.data_ptr(), B, H, dh, out.data_ptr(), st), "blk_fwd"),
                "block_bwd": lambda: chk(lib.mirec_attention_varlen_bwd(
                    qkv.data_ptr(), dout.data_ptr(), offs.data_ptr(), B, H, dh,
                    dqkv.data_ptr(), st), "blk_bwd"),
                "blockord_fwd": lambda: chk(lib.mirec_attention_ordered_fwd(
                    qkv.data_ptr(), offs.data_ptr(), order.data_ptr(), B, H, dh, out.data_ptr(),
                    st), "blko_fwd"),
                "blockord_bwd": lambda: chk(lib.mirec_attention_ordered_bwd(
                    qkv.data_ptr(), dout.data_ptr(), offs.data_ptr(), order.data_ptr(), B, H, dh,
                    dqkv.data_ptr(), st), "blko_bwd"),
                "packed_bwd": lambda: chk(lib.mirec_attention_packed_bwd(
                    qkv.data_ptr(), dout.data_ptr(), offs.data_ptr(), order[bp:].data_ptr(), B, H,
                    dh, dqkv.data_ptr(), n, st), "packed_bwd"),
                "packed_lse_bwd": lambda: chk(lib.mirec_attention_packed_bwd_lse(
                    qkv.data_ptr(), lse.data_ptr(), dout.data_ptr(), offs.data_ptr(),
                    order[bp:].data_ptr(), B, H, dh, dqkv.data_ptr(), n, st), "packed_lse_bwd"),
            }
            for name, fn in runs.items():
                if name in ("wave_bwd", "packed_lse_bwd"):
                    runs["wave_fwd"]()  # the forward's out / lse
                us = timed(fn, a.reps)
                by = by_b if name.endswith("bwd") else by_f
                print(json.dumps({"kernel": name, "order": a.order, "mix": mix, "B": B, "n_tok": n, "us": round(us, 1),
                                  "GBps": round(by / us / 1e3, 1),
                                  "tflops": round((10 if name.endswith("bwd") else 4) * t2 * dh * H
                                                  / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
