"""nn.Linear on token rows: f32 MFMA GEMMs (csrc/gemm.hip) for the forward,
the input gradient and the weight + bias gradient.

The packed SASRec / GraphSAGE activations are tall and thin (tens of
thousands of rows x d = 128..384).  mirec_gemm_nt computes y = x Wᵀ + b,
mirec_gemm_nn_ex dX = dY W (W read as stored); mirec_gemm_tn computes
dW = dYᵀ X and db = Σ dY in one pass over dY, cutting the long row reduction
into slices summed in a fixed order.  Shapes the kernels do not take (a
width not a multiple of 32 / 128) go to torch's GEMMs, where the weight
gradient is split over 32 row slices (one batched GEMM + a sum): the
library GEMM for dYᵀ X runs ~4x below its forward rate when the reduction
dimension is the long one (tools/gemm_forms.py).  Same parameters and
state_dict keys as nn.Linear.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import check, lib

SPLIT = 32
MIN_ROWS_PER_SLICE = 256
# MIREC_GEMM=0 routes every Linear through torch's GEMMs (A/B timing)
USE_MIREC_GEMM = os.environ.get("MIREC_GEMM", "1") != "0"
FORCE_MIREC_GEMM = False  # tests: every eligible shape on the mirec kernels


def _aligned(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
               and t.data_ptr() % 16 == 0 for t in ts)


def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None):
    """a [n, Kr] · b[No, Kr]ᵀ (+ bias) on mirec_gemm_nt, or None if the
    shapes are not the kernel's (Kr % 32, No % 128)."""
    n, kr = a.shape
    no = b.shape[0]
    if not (USE_MIREC_GEMM and kr % 32 == 0 and no % 128 == 0 and b.shape[1] == kr
            and _aligned(a, b) and (bias is None or _aligned(bias))):
        return None
    c = torch.empty(n, no, dtype=a.dtype, device=a.device)
    check(lib.mirec_gemm_nt(a.data_ptr(), b.data_ptr(), 0 if bias is None else bias.data_ptr(),
                            c.data_ptr(), n, kr, no, _lib.stream_handle()), "gemm_nt")
    return c


def gemm_nn(a: torch.Tensor, b: torch.Tensor):
    """a [n, Kr] · b [Kr, No] on mirec_gemm_nn_ex (b as stored: the weight of
    dX = dY W), or None if the shapes are not the kernel's."""
    n, kr = a.shape
    no = b.shape[1]
    if not (USE_MIREC_GEMM and kr % 32 == 0 and no % 128 == 0 and b.shape[0] == kr
            and _aligned(a, b)):
        return None
    c = torch.empty(n, no, dtype=a.dtype, device=a.device)
    check(lib.mirec_gemm_nn_ex(a.data_ptr(), None, b.data_ptr(), c.data_ptr(), None, 0, n, kr, no,
                               _lib.stream_handle()), "gemm_nn")
    return c


def gemm_tn(a: torch.Tensor, b: torch.Tensor, colsum: bool):
    """(a[n, M]ᵀ b[n, No], Σ_rows a or None) on mirec_gemm_tn, or None if
    the shapes are not the kernel's (M % 128, No % 128)."""
    n, m = a.shape
    no = b.shape[1]
    if not (USE_MIREC_GEMM and m % 128 == 0 and no % 128 == 0 and b.shape[0] == n
            and _aligned(a, b)):
        return None
    c = torch.empty(m, no, dtype=a.dtype, device=a.device)
    cs = torch.empty(m, dtype=a.dtype, device=a.device) if colsum else None
    work = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, m, no)), dtype=a.dtype,
                       device=a.device)
    check(lib.mirec_gemm_tn(a.data_ptr(), b.data_ptr(), c.data_ptr(),
                            0 if cs is None else cs.data_ptr(), n, m, no, work.data_ptr(),
                            _lib.stream_handle()), "gemm_tn")
    return c, cs


# MIREC_TORCH_COLSUM=1: torch's sum(0) instead (the round-3 form of the
# captured data-parallel step, kept to reproduce DESIGN.md §9.2)
_TORCH_COLSUM = os.environ.get("MIREC_TORCH_COLSUM", "0") == "1"


def col_sums(a: torch.Tensor) -> torch.Tensor:
    """Σ over the rows of a contiguous [n, m] float32 tensor, in a fixed order
    (mirec_col_sums: deterministic, capturable, and — up to n = 64 x 2048 /
    ceil(m / 256) rows — bitwise the same with zero rows appended, so the
    captured SASRec step, which sums over its token capacity, gives the eager
    step's bias gradients; torch's sum(0) picks its reduction tree from the
    row count: DESIGN.md §9.2).
    Tensors off the HIP device or not float32 (the module used as a plain
    nn.Linear, e.g. float64 on the host) take torch's sum."""
    if not (a.is_cuda and a.dtype == torch.float32) or _TORCH_COLSUM:
        return a.sum(0)
    a = a.contiguous()
    n, m = a.shape
    out = torch.empty(m, dtype=a.dtype, device=a.device)
    work = torch.empty(max(int(lib.mirec_col_sums_work_floats(n, m)), 1), dtype=a.dtype,
                       device=a.device)
    check(lib.mirec_col_sums(a.data_ptr(), n, m, out.data_ptr(), work.data_ptr(),
                             _lib.stream_handle()), "col_sums")
    return out


def weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dyᵀ x for dy [n, N], x [n, K] (contiguous rows), torch GEMMs (the
    slices' products summed by col_sums)."""
    n = dy.shape[0]
    if n < SPLIT * MIN_ROWS_PER_SLICE:
        return dy.t() @ x
    m = n // SPLIT
    main = SPLIT * m
    parts = torch.bmm(dy[:main].view(SPLIT, m, dy.shape[1]).transpose(1, 2),
                      x[:main].view(SPLIT, m, x.shape[1]))
    g = col_sums(parts.view(SPLIT, -1)).view(dy.shape[1], x.shape[1])
    if main < n:
        g = g + dy[main:].t() @ x[main:]
    return g


class _LinearSplitK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        x2 = x.reshape(-1, x.shape[-1])
        y = gemm_nt(x2, w, b) if x2.is_contiguous() else None
        if y is None:
            return F.linear(x, w, b)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        need = ctx.needs_input_grad
        dx = dw = db = None
        if need[0]:
            dx = gemm_nn(dy2, w)
            dx = (dy2 @ w if dx is None else dx).view(shape)
        want_db = ctx.has_bias and need[2]
        if need[1]:
            r = gemm_tn(dy2, x2, want_db)
            if r is None:
                dw = weight_grad(dy2, x2)
            else:
                dw, db = r
        if want_db and db is None:
            db = col_sums(dy2)
        return dx, dw, db


class _SageLinear(torch.autograd.Function):
    """y = act(x_self W[:, :d]ᵀ + x_nbr W[:, d:]ᵀ + b), the GraphSAGE hop's
    Linear over [x_self ; aggr] (model/graphsage.py:314-315) without the
    concatenation: the GEMM reads its A rows from the two tensors
    (mirec_gemm_nt_ex), adds the bias and applies the ReLU in its epilogue.
    Backward: the ReLU mask is applied to dY as it is loaded; dX = dY' W is
    written straight into the two input gradients (output split at d) and
    dW = dY'ᵀ [x_self | x_nbr], db = Σ dY' in one pass (mirec_gemm_tn_ex)."""

    @staticmethod
    def forward(ctx, xs, xn, w, b, relu: bool):
        n, d = xs.shape
        no = w.shape[0]
        y = torch.empty(n, no, dtype=xs.dtype, device=xs.device)
        check(lib.mirec_gemm_nt_ex(xs.data_ptr(), xn.data_ptr(), d, None, w.data_ptr(),
                                   _lib.ptr(b), y.data_ptr(), None, 0, int(relu), n, 2 * d, no,
                                   _lib.stream_handle()), "gemm_nt_ex")
        ctx.save_for_backward(xs, xn, w, y if relu else None)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, xn, w, y = ctx.saved_tensors
        n, d = xs.shape
        no = w.shape[0]
        dy = dy.contiguous()
        st = _lib.stream_handle()
        mask = _lib.ptr(y)
        dxs = torch.empty_like(xs)
        dxn = torch.empty_like(xn)
        check(lib.mirec_gemm_nn_ex(dy.data_ptr(), mask, w.data_ptr(), dxs.data_ptr(),
                                   dxn.data_ptr(), d, n, no, 2 * d, st), "gemm_nn_ex(dX)")
        dw = torch.empty_like(w)
        db = torch.empty(no, dtype=w.dtype, device=w.device) if ctx.has_bias else None
        work = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, no, 2 * d)), dtype=w.dtype,
                           device=w.device)
        check(lib.mirec_gemm_tn_ex(dy.data_ptr(), mask, xs.data_ptr(), xn.data_ptr(), d,
                                   dw.data_ptr(), _lib.ptr(db), n, no, 2 * d, work.data_ptr(), st),
              "gemm_tn_ex(dW)")
        return dxs, dxn, dw, db, None


def sage_linear(xs: torch.Tensor, xn: torch.Tensor, w: torch.Tensor,
                b: torch.Tensor | None, relu: bool) -> torch.Tensor:
    """act(Linear([xs ; xn])) for the GraphSAGE hop; the fused GEMMs when the
    shapes are theirs (d % 128, out % 128, aligned contiguous rows), else
    concatenation + Linear + ReLU."""
    d = xs.shape[1]
    if (USE_MIREC_GEMM and xs.dim() == 2 and xn.shape == xs.shape and d % 128 == 0
            and w.shape[1] == 2 * d and w.shape[0] % 128 == 0
            and _aligned(xs, xn, w) and (b is None or _aligned(b))):
        return _SageLinear.apply(xs, xn, w, b, bool(relu))
    y = _LinearSplitK.apply(torch.cat([xs, xn], dim=1), w, b)
    return y.relu() if relu else y


class _LinearReLU(torch.autograd.Function):
    """relu(x Wᵀ + b) with the bias and ReLU in the GEMM epilogue
    (mirec_gemm_nt_ex); backward: the ReLU mask applied to dY as it is loaded
    by dX = dY' W (mirec_gemm_nn_ex) and by dW = dY'ᵀ x, db = Σ dY'
    (mirec_gemm_tn_ex) — no elementwise kernels either way."""

    @staticmethod
    def forward(ctx, x, w, b):
        n, k = x.shape
        no = w.shape[0]
        y = torch.empty(n, no, dtype=x.dtype, device=x.device)
        check(lib.mirec_gemm_nt_ex(x.data_ptr(), None, 0, None, w.data_ptr(), _lib.ptr(b),
                                   y.data_ptr(), None, 0, 1, n, k, no, _lib.stream_handle()),
              "gemm_nt_ex(relu)")
        ctx.save_for_backward(x, w, y)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        n, k = x.shape
        no = w.shape[0]
        dy = dy.contiguous()
        st = _lib.stream_handle()
        dx = torch.empty_like(x)
        check(lib.mirec_gemm_nn_ex(dy.data_ptr(), y.data_ptr(), w.data_ptr(), dx.data_ptr(), None,
                                   0, n, no, k, st), "gemm_nn_ex(relu dX)")
        dw = torch.empty_like(w)
        db = torch.empty(no, dtype=w.dtype, device=w.device) if ctx.has_bias else None
        work = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, no, k)), dtype=w.dtype,
                           device=w.device)
        check(lib.mirec_gemm_tn_ex(dy.data_ptr(), y.data_ptr(), x.data_ptr(), None, 0,
                                   dw.data_ptr(), _lib.ptr(db), n, no, k, work.data_ptr(), st),
              "gemm_tn_ex(relu dW)")
        return dx, dw, db


def linear_relu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """relu(F.linear(x, w, b)) — fused on the mirec GEMMs when the shapes are
    theirs (2-D aligned contiguous x, in and out widths multiples of 128)."""
    if (USE_MIREC_GEMM and x.dim() == 2 and x.shape[1] % 128 == 0 and w.shape[0] % 128 == 0
            and _aligned(x, w) and (b is None or _aligned(b))):
        return _LinearReLU.apply(x, w, b)
    return _LinearSplitK.apply(x, w, b).relu()


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    return _LinearSplitK.apply(x, w, b)


class Linear(nn.Linear):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _LinearSplitK.apply(x, self.weight, self.bias)


@contextlib.contextmanager
def blas_backend(name: str | None):
    """Temporarily select torch's BLAS backend ("cublas" = rocBLAS,
    "cublaslt" = hipBLASLt on ROCm).  rocBLAS launches small GEMMs with
    about half the host cost (8.5 vs 19 us per call, tools/gemm_forms.py),
    which decides the step time of launch-bound models (SASRec)."""
    if not name:
        yield
        return
    prev = torch.backends.cuda.preferred_blas_library()
    torch.backends.cuda.preferred_blas_library(name)
    try:
        yield
    finally:
        torch.backends.cuda.preferred_blas_library(prev)
