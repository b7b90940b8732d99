"""Debug: mirec_gemm_resnorm repeated on fixed inputs (bitwise repeatability
of out / y / mean / rstd) at ragged and aligned row counts."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from furusato_recommend_amd import _lib
lib, st, check = _lib.lib, _lib.stream_handle(), _lib.check
REPS = int(os.environ.get("REPS", "20"))
d = 128
for n in (56321, 56320, 20000):
    for k in (128, 256):
        torch.manual_seed(n + k)
        x = torch.randn(n, k, device="cuda"); w = torch.randn(d, k, device="cuda") * k ** -0.5
        res = torch.randn(n, d, device="cuda"); bias = torch.randn(d, device="cuda") * 0.1
        gam = torch.rand(d, device="cuda") + 0.5; bet = torch.randn(d, device="cuda") * 0.1
        first, nd = None, 0
        for rep in range(REPS):
            out = torch.empty(n, d, device="cuda"); y = torch.empty_like(out)
            mean = torch.empty(n, device="cuda"); rstd = torch.empty_like(mean)
            check(lib.mirec_gemm_resnorm(x.data_ptr(), w.data_ptr(), n, k, d, res.data_ptr(),
                                         bias.data_ptr(), gam.data_ptr(), bet.data_ptr(), 1, 0.0, 0,
                                         None, 1e-5, out.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                         rstd.data_ptr(), st), "gemm_resnorm")
            cur = (out, y, mean, rstd)
            if first is None:
                first = cur
            elif not all(torch.equal(a, b) for a, b in zip(cur, first)):
                nd += 1
        torch.cuda.synchronize()
        print(f"  lib={os.path.basename(_lib.LIB_PATH)} gemm_resnorm n={n} k={k}: {nd}/{REPS - 1} runs differ", flush=True)
