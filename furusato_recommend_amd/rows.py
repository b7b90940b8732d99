"""Row gather with an atomic scatter-add backward (libmirec): the embedding
lookup of the GraphSAGE hop path and of SASRec's sequence / item inputs.

``gather_rows(table, ids)`` = ``table[ids]`` with ids < 0 giving zero rows
(and no gradient).  Its backward adds each gradient row into the table
gradient with float atomics (one 256-B wave instruction per 64 floats), in
place of torch's sort-based embedding/index backward.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check, lib


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, ids):
        n, d = ids.numel(), table.shape[1]
        out = torch.empty(n, d, dtype=table.dtype, device=table.device)
        check(lib.mirec_gather_rows(table.data_ptr(), ids.data_ptr(), n, d, out.data_ptr(),
                                    _lib.stream_handle()), "gather_rows")
        ctx.save_for_backward(ids)
        ctx.shape = table.shape
        return out

    @staticmethod
    def backward(ctx, grad):
        (ids,) = ctx.saved_tensors
        g = torch.zeros(ctx.shape, dtype=grad.dtype, device=grad.device)
        check(lib.mirec_scatter_add_rows(grad.contiguous().data_ptr(), ids.data_ptr(),
                                         ids.numel(), ctx.shape[1], g.data_ptr(),
                                         _lib.stream_handle()), "scatter_add_rows")
        return g, None


def gather_rows(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """table[ids] for int32 ids of any shape (-1 = zero row); differentiable
    w.r.t. ``table``.  Returns [*ids.shape, table.shape[1]]."""
    if table.dtype != torch.float32 or table.dim() != 2 or table.shape[1] % 4:
        raise ValueError("gather_rows: float32 [n, d] table with d % 4 == 0")
    flat = ids.reshape(-1).to(torch.int32).contiguous()
    out = _GatherRows.apply(table.contiguous(), flat)
    return out.view(*ids.shape, table.shape[1])


def slice_norms(table: torch.Tensor, split_rows: int):
    """(‖table[:split_rows]‖₂, ‖table[split_rows:]‖₂) as 0-d tensors, one
    pass over the table (mirec_slice_norms; fixed summation order)."""
    norms = slice_norms2(table, split_rows)
    return norms[0], norms[1]


def slice_norms2(table: torch.Tensor, split_rows: int) -> torch.Tensor:
    """The two slice norms as one [2] tensor."""
    if not (table.is_cuda and table.dtype == torch.float32 and table.is_contiguous()
            and table.shape[-1] % 4 == 0):
        raise ValueError("slice_norms: contiguous float32 table with rows of 4k floats")
    norms = torch.empty(2, dtype=table.dtype, device=table.device)
    work = torch.empty(int(lib.mirec_slice_norms_work_floats()), dtype=table.dtype,
                       device=table.device)
    check(lib.mirec_slice_norms(table.data_ptr(), table.numel(), split_rows * table.shape[-1],
                                work.data_ptr(), norms.data_ptr(), _lib.stream_handle()),
          "slice_norms")
    return norms


class _GatherRowsNorm(torch.autograd.Function):
    """(table[ids], ‖table‖₂) as one autograd node: the embedding lookup and
    the embedding-norm term of the SASRec loss (model/sasrec.py:423-435) both
    differentiate into the same table gradient, which the backward writes
    once — (g_norm / ‖table‖) · table (0 when the norm is 0, as torch's
    norm backward) — and then scatter-adds the row gradients into, instead of
    two table-sized gradients added by autograd."""

    @staticmethod
    def forward(ctx, table, ids):
        n, d = ids.numel(), table.shape[1]
        out = torch.empty(n, d, dtype=table.dtype, device=table.device)
        check(lib.mirec_gather_rows(table.data_ptr(), ids.data_ptr(), n, d, out.data_ptr(),
                                    _lib.stream_handle()), "gather_rows")
        norm = slice_norms(table, table.shape[0])[0]
        ctx.save_for_backward(table, ids, norm)
        return out, norm

    @staticmethod
    def backward(ctx, grad, g_norm):
        table, ids, norm = ctx.saved_tensors
        if g_norm is None:
            g = torch.zeros_like(table)
        else:
            scale = torch.where(norm > 0, g_norm / norm, torch.zeros_like(norm))
            g = table * scale
        if grad is not None:
            check(lib.mirec_scatter_add_rows(grad.contiguous().data_ptr(), ids.data_ptr(),
                                             ids.numel(), table.shape[1], g.data_ptr(),
                                             _lib.stream_handle()), "scatter_add_rows")
        return g, None


def gather_rows_norm(table: torch.Tensor, ids: torch.Tensor):
    """(gather_rows(table, ids), table.norm(2)) with one fused backward."""
    if table.dtype != torch.float32 or table.dim() != 2 or table.shape[1] % 4:
        raise ValueError("gather_rows_norm: float32 [n, d] table with d % 4 == 0")
    flat = ids.reshape(-1).to(torch.int32).contiguous()
    out, norm = _GatherRowsNorm.apply(table.contiguous(), flat)
    return out.view(*ids.shape, table.shape[1]), norm
