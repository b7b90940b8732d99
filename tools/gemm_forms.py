"""Times equivalent formulations of the SASRec Linear GEMMs (f32) to pick the
hipBLASLt problem orientation that runs fastest (C4 shapes: n packed tokens,
d = 128, in_proj N = 384)."""
import torch


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


def main():
    n, K = 56_320, 128
    for N in (384, 128):
        x = torch.randn(n, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        dy = torch.randn(n, N, device="cuda")
        fl = 2.0 * n * K * N
        res = {
            "fwd F.linear": t(lambda: torch.nn.functional.linear(x, w, b)),
            "fwd x@w.t()": t(lambda: x @ w.t()),
            "fwd (w@x.t()).t()": t(lambda: (w @ x.t()).t()),
            "fwd addmm": t(lambda: torch.addmm(b, x, w.t())),
            "dX dy@w": t(lambda: dy @ w),
            "dX (w.t()@dy.t()).t()": t(lambda: (w.t() @ dy.t()).t()),
            "dW dy.t()@x": t(lambda: dy.t() @ x),
            "dW (x.t()@dy).t()": t(lambda: (x.t() @ dy).t()),
            "dW chunked4": t(lambda: sum(dy[i::4].t() @ x[i::4] for i in range(4))),
        }
        for S in (4, 8, 16, 32, 64, 128):
            res[f"dW bmm split{S}"] = t(lambda S=S: torch.bmm(
                dy.view(S, n // S, N).transpose(1, 2), x.view(S, n // S, K)).sum(0))
        print(f"N={N}", {k: f"{v:.1f}us {fl / v / 1e6:.1f}TF" for k, v in res.items()})


if __name__ == "__main__":
    main()
