"""Error of the split-bf16 GEMMs vs torch fp32 matmul, both against float64,
per element relative to its scale sum_k |a_ik b_kj|, on operands spanning
twelve decades (the data of test_gemm_split_bf16_is_f32_accurate) and on
plain N(0, 1) operands.  One JSON line per (form, shape, data)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from furusato_recommend_amd import linear as LN
    from furusato_recommend_amd.linear import gemm_nn, gemm_nt
    LN.FORCE_MIREC_GEMM = True
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(5)
    for data in ("wide", "normal"):
        for n, k, m in ((4096, 128, 384), (20_000, 384, 128), (4096, 4096, 512)):
            sa = 10 ** (12 * torch.rand(n, 1, device="cuda") - 6) if data == "wide" else 1.0
            sb = 10 ** (12 * torch.rand(m, 1, device="cuda") - 6) if data == "wide" else 1.0
            a = torch.randn(n, k, device="cuda") * sa
            b = torch.randn(m, k, device="cuda") * sb
            scale = a.double().abs() @ b.double().abs().t()
            ref = a.double() @ b.double().t()

            def err(c):
                e = (c.double() - ref).abs() / scale
                return float(e.max()), float(e.mean())
            line = {"data": data, "n": n, "k": k, "m": m, "torch_fp32": err(a @ b.t()),
                    "split_nt": err(gemm_nt(a, b)), "split_nn": err(gemm_nn(a, b.t().contiguous()))}
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
