"""Device time of the f32 MFMA GEMMs (csrc/gemm.hip) on the shapes of the C3
(GraphSAGE [25,10] d=128) and C4 (SASRec d=128) steps, against the f32
matrix peak (157.3 TF, MI355X_MICROARCH.md).  One JSON line per shape.
MIREC_LIB selects a library build (A/B of kernel variants).

    python tools/gemm_bench.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = 157.3


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
    a = ap.parse_args()
    from furusato_recommend_amd import _lib
    lib, st = _lib.lib, _lib.stream_handle()
    chk = _lib.check
    dev = "cuda"
    out = []

    def nt(name, n, kr, no, dual=False, mask=False, relu=False, split=False):
        A = torch.randn(n, kr, device=dev)
        A1, A2 = (A[:, : kr // 2].contiguous(), A[:, kr // 2:].contiguous()) if dual else (A, None)
        B = torch.randn(no, kr, device=dev) * 0.05
        bias = torch.randn(no, device=dev)
        M = torch.randn(n, kr, device=dev) if mask else None
        C = torch.empty(n, no if not split else no // 2, device=dev)
        C2 = torch.empty(n, no // 2, device=dev) if split else None
        def f():
            chk(lib.mirec_gemm_nt_ex(A1.data_ptr(), _lib.ptr(A2), kr // 2 if dual else 0,
                                     _lib.ptr(M), B.data_ptr(), None if mask else bias.data_ptr(),
                                     C.data_ptr(), _lib.ptr(C2), no // 2 if split else 0,
                                     int(relu), n, kr, no, st), name)
        us = timed(f, a.reps)
        tf = 2.0 * n * kr * no / us / 1e6
        out.append({"gemm": name, "kind": "nt", "n": n, "K": kr, "N": no, "us": round(us, 1),
                    "tflops": round(tf, 1), "frac_peak": round(tf / PEAK_TF, 3)})

    def nn(name, n, kr, no, mask=False, split=False):
        A = torch.randn(n, kr, device=dev)
        B = torch.randn(kr, no, device=dev) * 0.05
        M = torch.randn(n, kr, device=dev) if mask else None
        C = torch.empty(n, no if not split else no // 2, device=dev)
        C2 = torch.empty(n, no // 2, device=dev) if split else None
        def f():
            chk(lib.mirec_gemm_nn_ex(A.data_ptr(), _lib.ptr(M), B.data_ptr(), C.data_ptr(),
                                     _lib.ptr(C2), no // 2 if split else 0, n, kr, no, st), name)
        us = timed(f, a.reps)
        tf = 2.0 * n * kr * no / us / 1e6
        out.append({"gemm": name, "kind": "nn", "n": n, "K": kr, "N": no, "us": round(us, 1),
                    "tflops": round(tf, 1), "frac_peak": round(tf / PEAK_TF, 3)})

    def tn(name, n, m, no, dual=False, mask=False):
        A = torch.randn(n, m, device=dev)
        Bf = torch.randn(n, no, device=dev)
        B1, B2 = (Bf[:, : no // 2].contiguous(), Bf[:, no // 2:].contiguous()) if dual else (Bf, None)
        M = torch.randn(n, m, device=dev) if mask else None
        C = torch.empty(m, no, device=dev)
        cs = torch.empty(m, device=dev)
        work = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, m, no)), device=dev)
        def f():
            chk(lib.mirec_gemm_tn_ex(A.data_ptr(), _lib.ptr(M), B1.data_ptr(), _lib.ptr(B2),
                                     no // 2 if dual else 0, C.data_ptr(), cs.data_ptr(), n, m, no,
                                     work.data_ptr(), st), name)
        us = timed(f, a.reps)
        tf = 2.0 * n * m * no / us / 1e6
        out.append({"gemm": name, "kind": "tn", "n": n, "M": m, "N": no, "us": round(us, 1),
                    "tflops": round(tf, 1), "frac_peak": round(tf / PEAK_TF, 3)})

    nt("c3_small_fwd", 6144, 256, 128, dual=True, relu=True)
    n3 = 153_600
    nt("c3_l0_fwd", n3, 256, 128, dual=True, relu=True)
    nt("c3_l0_dx", n3, 128, 256, mask=True, split=True)
    nn("c3_l0_dx_nn", n3, 128, 256, mask=True, split=True)
    tn("c3_l0_dw", n3, 128, 256, dual=True, mask=True)
    n4 = 56_320
    nt("c4_qkv_fwd", n4, 128, 384)
    nt("c4_proj_fwd", n4, 128, 128)
    nt("c4_qkv_dx", n4, 384, 128)
    nn("c4_qkv_dx_nn", n4, 384, 128)
    nn("c4_proj_dx_nn", n4, 128, 128)
    tn("c4_qkv_dw", n4, 384, 128)
    tn("c4_proj_dw", n4, 128, 128)
    nt("sq_4096", 4096, 4096, 4096)
    for line in out:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
