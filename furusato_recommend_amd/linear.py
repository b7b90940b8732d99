"""nn.Linear with a split-K weight gradient.

On the packed SASRec / GraphSAGE activations (tens of thousands of rows,
d = 128) the library GEMM for dW = dYᵀ X (a reduction over every row) runs
at ~20 TFLOP/s f32, 4x below the forward GEMMs of the same size: the
reduction dimension is the long one.  Cutting the rows into 32 slices, one
batched GEMM over the slices and a sum of the 32 partial [N, K] products
runs at 60-85 TFLOP/s (measured on MI355X, tools/gemm_forms.py).  Same
parameters and state_dict keys as nn.Linear; the forward is unchanged.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F

SPLIT = 32
MIN_ROWS_PER_SLICE = 256


def weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dyᵀ x for dy [n, N], x [n, K] (contiguous rows)."""
    n = dy.shape[0]
    if n < SPLIT * MIN_ROWS_PER_SLICE:
        return dy.t() @ x
    m = n // SPLIT
    main = SPLIT * m
    g = torch.bmm(dy[:main].view(SPLIT, m, dy.shape[1]).transpose(1, 2),
                  x[:main].view(SPLIT, m, x.shape[1])).sum(0)
    if main < n:
        g = g + dy[main:].t() @ x[main:]
    return g


class _LinearSplitK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx = (dy2 @ w).view(shape) if ctx.needs_input_grad[0] else None
        dw = weight_grad(dy2, x2.contiguous()) if ctx.needs_input_grad[1] else None
        db = dy2.sum(0) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        return dx, dw, db


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
