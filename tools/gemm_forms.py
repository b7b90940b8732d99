"""SASRec Linear GEMMs (f32): device time of equivalent formulations and the
host-side cost per call of each BLAS backend torch can use on ROCm."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, reps=20):
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


def host_us(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / reps * 1e6


def main():
    n, K, N = 56_320, 128, 384
    x = torch.randn(n, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    dy = torch.randn(n, N, device="cuda")
    xs, ws = torch.randn(64, K, device="cuda"), torch.randn(N, K, device="cuda")
    from furusato_recommend_amd.linear import gemm_nt, gemm_tn
    wt = w.t().contiguous()
    for (nn_, kk, NN) in ((n, K, N), (n, K, K)):
        xa, wa, ba = torch.randn(nn_, kk, device="cuda"), torch.randn(NN, kk, device="cuda"), \
            torch.randn(NN, device="cuda")
        dya = torch.randn(nn_, NN, device="cuda")
        wta = wa.t().contiguous()
        fl = 2.0 * nn_ * kk * NN
        r = {"fwd": t(lambda: gemm_nt(xa, wa, ba)), "dX": t(lambda: gemm_nt(dya, wta)),
             "dW+db": t(lambda: gemm_tn(dya, xa, True)),
             "torch fwd": t(lambda: torch.addmm(ba, xa, wa.t())),
             "torch dX": t(lambda: dya @ wa),
             "torch dW split32 + db": t(lambda: (torch.bmm(
                 dya.view(32, nn_ // 32, NN).transpose(1, 2), xa.view(32, nn_ // 32, kk)).sum(0),
                 dya.sum(0)))}
        print(f"mirec gemm n={nn_} K={kk} N={NN}:",
              {k_: f"{v:.1f} us {fl / v / 1e6:.0f} TF/s" for k_, v in r.items()}, flush=True)
    for lib in ("default", "cublaslt", "cublas"):
        try:
            if lib != "default":
                torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            print(lib, "unavailable", e)
            continue
        res = {
            "addmm dev us": t(lambda: torch.addmm(b, x, w.t())),
            "dX mm dev us": t(lambda: dy @ w),
            "dW split32 dev us": t(lambda: torch.bmm(dy.view(32, n // 32, N).transpose(1, 2),
                                                     x.view(32, n // 32, K)).sum(0)),
            "small mm host us": host_us(lambda: xs @ ws.t()),
            "small addmm host us": host_us(lambda: torch.addmm(b, xs, ws.t())),
            "small bmm host us": host_us(lambda: torch.bmm(xs.view(4, 16, K), ws.t().expand(4, K, N))),
        }
        print(lib, torch.backends.cuda.preferred_blas_library(),
              {k: round(v, 1) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
