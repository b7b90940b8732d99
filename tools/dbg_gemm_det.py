"""Debug: repeat each mirec GEMM form many times on fixed inputs; count
results that differ from the first run / from float64."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from furusato_recommend_amd.linear import gemm_nt, gemm_nn, gemm_tn
from furusato_recommend_amd import linear as LN
LN.FORCE_MIREC_GEMM = True
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 30


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


for name, fn, shapes in (
        ("nt", lambda a, b: gemm_nt(a, b), [(153601, 128, 128)]),
        ("nn", lambda a, b: gemm_nn(a, b.t().contiguous()), [(153600, 128, 128), (153601, 128, 128), (153601, 384, 128)]),
        ("tn", lambda a, b: gemm_tn(a, b, True)[0], []) ):
    for n, k, m in shapes:
        torch.manual_seed(n + k + m)
        if name == "tn":
            a = torch.randn(n, k, device="cuda"); b = torch.randn(n, m, device="cuda")
            ref = a.double().t() @ b.double()
        else:
            a = torch.randn(n, k, device="cuda"); b = torch.randn(m, k, device="cuda")
            ref = a.double() @ b.double().t()
        c0 = fn(a, b)
        ndiff, worst = 0, rel(c0, ref)
        for _ in range(REPS):
            c = fn(a, b)
            if not torch.equal(c, c0):
                ndiff += 1
            worst = max(worst, rel(c, ref))
        torch.cuda.synchronize()
        print(f"{name} n={n} k={k} m={m}: {ndiff}/{REPS} runs differ from the first; worst rel vs f64 {worst:.1e}", flush=True)
