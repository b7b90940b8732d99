"""Debug: per-leaf gradient agreement of the fused SASRec block tail vs the
two-node path (and a float64 torch chain without dropout)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from furusato_recommend_amd import sasrec as S


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


d = 128
names = ["o", "res", "w_o", "w_f", "b_o", "b_f", "lnf_w", "lnf_b", "lnn_w", "lnn_b"]
for has_next in (True, False):
    for n in (1, 777, 56321):
        for p in (0.2, 0.0):
            torch.manual_seed(n)
            o = torch.randn(n, d, device="cuda", requires_grad=True)
            res = torch.randn(n, d, device="cuda", requires_grad=True)
            w_o = (torch.randn(d, d, device="cuda") * d ** -0.5).requires_grad_(True)
            w_f = (torch.randn(d, d, device="cuda") * d ** -0.5).requires_grad_(True)
            b_o = (torch.randn(d, device="cuda") * 0.1).requires_grad_(True)
            b_f = (torch.randn(d, device="cuda") * 0.1).requires_grad_(True)
            ln_f = torch.nn.LayerNorm(d, device="cuda")
            ln_n = torch.nn.LayerNorm(d, device="cuda") if has_next else None
            with torch.no_grad():
                for ln in (ln_f, ln_n):
                    if ln is not None:
                        ln.weight.uniform_(0.5, 1.5)
                        ln.bias.uniform_(-0.2, 0.2)
            outs = []
            for fuse in (True, False):
                S.FUSE_BLOCK_TAIL = fuse
                torch.manual_seed(11)
                outs.append(S.block_tail(o, res, w_o, b_o, ln_f, w_f, b_f, ln_n, p=p))
            S.FUSE_BLOCK_TAIL = True
            g_r = torch.randn(n, d, device="cuda")
            g_y = torch.randn(n, d, device="cuda") if has_next else None
            leaves = [o, res, w_o, w_f, b_o, b_f, ln_f.weight, ln_f.bias] + (
                [ln_n.weight, ln_n.bias] if has_next else [])
            grads = []
            for r2, y2 in outs:
                ys, gs = [r2], [g_r]
                if has_next:
                    ys.append(y2)
                    gs.append(g_y)
                grads.append(torch.autograd.grad(ys, leaves, gs))
            line = " ".join(f"{nm}={rel(a, b):.1e}" for nm, a, b in zip(names, grads[0], grads[1]))
            print(f"next={has_next} n={n} p={p}: {line}", flush=True)
