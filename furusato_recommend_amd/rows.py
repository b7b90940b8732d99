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
    """(table[ids[:split]], table[ids[split:]], ‖table‖₂) as one autograd
    node: the embedding lookups and the embedding-norm term of the SASRec
    loss (model/sasrec.py:423-435) all differentiate into the same table
    gradient G = c·table + S, c = g_norm / ‖table‖ (0 when the norm is 0, as
    torch's norm backward), S = the row gradients scattered by id.  The two
    row groups arrive as separate gradients (no concatenation).
    With a ``sink`` (graphsage.TableGrad, one slice) the backward only sorts
    and sums S (mirec_table_grad_sorted, deterministic) and leaves c on the
    device: G is formed inside the table's Adam kernel (or materialised as
    .grad when sink.dense).  Without one it writes c·table and scatter-adds
    the rows with float atomics."""

    @staticmethod
    def forward(ctx, table, ids, split: int, sink, norm_in):
        n, d = ids.numel(), table.shape[1]
        out = torch.empty(n, d, dtype=table.dtype, device=table.device)
        check(lib.mirec_gather_rows(table.data_ptr(), ids.data_ptr(), n, d, out.data_ptr(),
                                    _lib.stream_handle()), "gather_rows")
        # the table's norm: given (kept from the last fused Adam) or one pass
        norm = slice_norms(table, table.shape[0])[0] if norm_in is None else norm_in.view(())
        ctx.save_for_backward(table, ids, norm)
        ctx.split, ctx.sink = split, sink
        ctx.set_materialize_grads(False)
        return out[:split], out[split:], norm

    @staticmethod
    def backward(ctx, g_a, g_b, g_norm):
        table, ids, norm = ctx.saved_tensors
        k, sink = ctx.split, ctx.sink
        st = _lib.stream_handle()
        parts = [(ids[:k], g_a), (ids[k:], g_b)]
        parts = [(i, g.contiguous()) for i, g in parts if g is not None and i.numel() > 0]
        if sink is not None:
            if g_norm is None:
                sink.coef.zero_()
            else:
                check(lib.mirec_norm_coef(g_norm.contiguous().data_ptr(), 0, norm.data_ptr(), 0,
                                          2, sink.coef.data_ptr(), st), "norm_coef")
            if parts:
                sink.accumulate([(i, g, 1, 0, 0.0, 0) for i, g in parts])
            else:
                sink.skip()
            return (sink.materialize(table) if sink.dense else None), None, None, None, None
        if g_norm is None:
            g = torch.zeros_like(table)
        else:
            scale = torch.where(norm > 0, g_norm / norm, torch.zeros_like(norm))
            g = table * scale
        for i, gr in parts:
            check(lib.mirec_scatter_add_rows(gr.data_ptr(), i.data_ptr(), i.numel(),
                                             table.shape[1], g.data_ptr(), st),
                  "scatter_add_rows")
        return g, None, None, None, None


def gather_rows_norm(table: torch.Tensor, ids: torch.Tensor, split: int | None = None,
                     sink=None, norm: torch.Tensor | None = None):
    """(gather_rows(table, ids), table.norm(2)) with one fused backward; with
    ``split`` the rows come back as the two groups ids[:split], ids[split:]
    ((rows_a, rows_b, norm)); ``sink``: see _GatherRowsNorm; ``norm``: the
    table's norm when the caller already holds it (a 1-element device
    tensor, read when the kernels run)."""
    if table.dtype != torch.float32 or table.dim() != 2 or table.shape[1] % 4:
        raise ValueError("gather_rows_norm: float32 [n, d] table with d % 4 == 0")
    flat = ids.reshape(-1).to(torch.int32).contiguous()
    k = flat.numel() if split is None else int(split)
    if not 0 <= k <= flat.numel():
        raise ValueError("gather_rows_norm: split outside the ids")
    a, b, norm = _GatherRowsNorm.apply(table.contiguous(), flat, k, sink, norm)
    if split is None:
        return a.view(*ids.shape, table.shape[1]), norm
    return a, b, norm

