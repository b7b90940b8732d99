"""Debug: mirec_gemm_nn_resnorm_bwd (fused) vs gemm_nn_ex + resnorm_bwd at
n = 56321, repeated, plus the GEMM part alone vs float64."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from furusato_recommend_amd import _lib
from furusato_recommend_amd.linear import gemm_nn
lib, st, check = _lib.lib, _lib.stream_handle(), _lib.check


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def P(t):
    return 0 if t is None else t.data_ptr()


d = 128
import os as _o
REPS = int(_o.environ.get('REPS', '3'))
for n in (56321, 56320, 20000):
    torch.manual_seed(n)
    A = torch.randn(n, d, device="cuda")
    W = torch.randn(d, d, device="cuda") * d ** -0.5
    out = torch.randn(n, d, device="cuda")
    mean = out.mean(1)
    rstd = (out.var(1, unbiased=False) + 1e-5).rsqrt()
    g_out = torch.randn(n, d, device="cuda")
    gamma = torch.rand(d, device="cuda") + 0.5
    gy_ref = A.double() @ W.double()
    gy = gemm_nn(A, W)
    res = []
    for rep in range(REPS):
        d_res = torch.empty(n, d, device="cuda"); d_z = torch.empty_like(d_res)
        work = torch.empty(int(lib.mirec_gemm_nn_resnorm_bwd_work_floats(n, d)), device="cuda")
        dg = torch.empty(d, device="cuda"); db = torch.empty(d, device="cuda"); dbias = torch.empty(d, device="cuda")
        check(lib.mirec_gemm_nn_resnorm_bwd(A.data_ptr(), W.data_ptr(), n, d, d, g_out.data_ptr(),
                                            out.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                            gamma.data_ptr(), 1, 0.0, 0, None, d_res.data_ptr(),
                                            d_z.data_ptr(), work.data_ptr(), dg.data_ptr(),
                                            db.data_ptr(), dbias.data_ptr(), st), "fused")
        res.append((d_res, d_z, dg, db, dbias))
    # unfused
    d_res2 = torch.empty(n, d, device="cuda"); d_z2 = torch.empty_like(d_res2)
    work2 = torch.empty(int(lib.mirec_resnorm_work_floats(n, d)), device="cuda")
    dg2 = torch.empty(d, device="cuda"); db2 = torch.empty(d, device="cuda"); dbias2 = torch.empty(d, device="cuda")
    check(lib.mirec_resnorm_bwd(gy.data_ptr(), g_out.data_ptr(), out.data_ptr(), mean.data_ptr(),
                                rstd.data_ptr(), gamma.data_ptr(), n, d, 1, 0.0, 0, None,
                                d_res2.data_ptr(), d_z2.data_ptr(), work2.data_ptr(),
                                dg2.data_ptr(), db2.data_ptr(), dbias2.data_ptr(), st), "unfused")
    torch.cuda.synchronize()
    print(f"n={n} gemm_nn vs f64 {rel(gy, gy_ref):.1e}", flush=True)
    nbad = sum(int(((a - d_res2).abs().max(1).values > 1e-4 * d_res2.abs().max()).sum() > 0) for a, *_ in res)
    print(f"  lib={_o.path.basename(_lib.LIB_PATH)} n={n}: {nbad}/{REPS} fused runs with a bad row", flush=True)
    shown = 0
    for rep, (a, b, c, e, f) in enumerate(res):
        diff = (a - d_res2).abs()
        rows = (diff.max(1).values > 1e-4 * d_res2.abs().max()).nonzero().flatten().tolist()
        for r in rows[:2]:
            if shown >= 4:
                break
            shown += 1
            cols = (diff[r] > 1e-4 * d_res2.abs().max()).nonzero().flatten().tolist()
            print(f"    rep{rep} row {r} (tile {r // 64}, local {r % 64}): {len(cols)} bad cols "
                  f"{cols[:12]} max diff {float(diff[r].max()):.3e}", flush=True)
    for rep, (a, b, c, e, f) in enumerate(res[:0]):
        bad = ((a - d_res2).abs().max(1).values > 1e-4 * d_res2.abs().max()).nonzero().flatten()
        print(f"  rep{rep}: d_res {rel(a, d_res2):.1e} d_z {rel(b, d_z2):.1e} dgamma {rel(c, dg2):.1e} "
              f"dbeta {rel(e, db2):.1e} dbias {rel(f, dbias2):.1e} bad_rows {bad.numel()} "
              f"first {bad[:8].tolist()} repeat_equal {torch.equal(a, res[0][0])}", flush=True)
