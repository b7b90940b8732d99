"""``torch.ops.mirec.*`` — the propagation hot path registered as PyTorch
operators (``torch.ops.mirec.lgcn_propagate(x, csr) -> y``
wrapped with its autograd formula), on top of the same C ABI
(``mirec_propagate``) the modules call.

Operator arguments must be tensors and scalars, so a graph (its CSR, the
normalisation and the hub-row split of ``graph.Graph``) is passed as an
integer handle: ``handle(graph)`` registers it (weakly: the entry goes when
the Graph object does) and returns the id.  The autograd node of a call keeps
the Graph object itself alive until the backward has run (a temporary
``LGConv()``, or one module called on a second edge_index before the first
call's backward, would otherwise drop the only other reference).

    h = ops.handle(graph)
    y = torch.ops.mirec.lgcn_propagate(x, h)          # y = Â x
    y.backward(g)                                      # x.grad = Âᵀ g

``lgcn_propagate_t`` is Âᵀ x (the same CSR for a symmetric edge multiset,
the transposed one otherwise).  Both have fake (meta) implementations, so
they trace under torch.compile / torch.export without running a kernel.
Reference call sites: model/lgcn.py:66,82 (``LGConv()(x, edge_index)``).
"""
from __future__ import annotations

import itertools
import weakref

import torch

_graphs: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()
_ids = itertools.count(1)


def handle(graph) -> int:
    """The operator handle of a graph.Graph (registered on first use)."""
    h = getattr(graph, "_op_handle", None)
    if h is None or _graphs.get(h) is not graph:
        h = next(_ids)
        _graphs[h] = graph
        graph._op_handle = h
    return h


def _graph(h: int):
    g = _graphs.get(int(h))
    if g is None:
        raise ValueError(f"mirec: no graph registered under handle {h}")
    return g


def _apply(g, x: torch.Tensor) -> torch.Tensor:
    from .lgconv import _spmm  # width padding / column blocks for any D
    if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 2:
        raise ValueError("mirec.lgcn_propagate: float32 [N, D] tensor on the HIP device")
    if x.shape[0] != g.n_nodes:
        raise ValueError(f"mirec.lgcn_propagate: x has {x.shape[0]} rows, graph {g.n_nodes}")
    return _spmm(g, x)


@torch.library.custom_op("mirec::lgcn_propagate", mutates_args=())
def lgcn_propagate(x: torch.Tensor, graph: int) -> torch.Tensor:
    """y = Â x on graph ``graph`` (csrc/prop.hip prop_kernel)."""
    return _apply(_graph(graph), x)


@torch.library.custom_op("mirec::lgcn_propagate_t", mutates_args=())
def lgcn_propagate_t(x: torch.Tensor, graph: int) -> torch.Tensor:
    """y = Âᵀ x (the backward of lgcn_propagate)."""
    g = _graph(graph)
    return _apply(g if g.symmetric else g.transpose, x)


@lgcn_propagate.register_fake
def _(x, graph):
    return torch.empty_like(x)


@lgcn_propagate_t.register_fake
def _(x, graph):
    return torch.empty_like(x)


def _setup(ctx, inputs, output):
    ctx.graph_obj = _graph(inputs[1])  # strong reference for the node's lifetime


def _bwd(ctx, grad):
    return torch.ops.mirec.lgcn_propagate_t(grad.contiguous(), handle(ctx.graph_obj)), None


def _bwd_t(ctx, grad):
    return torch.ops.mirec.lgcn_propagate(grad.contiguous(), handle(ctx.graph_obj)), None


lgcn_propagate.register_autograd(_bwd, setup_context=_setup)
lgcn_propagate_t.register_autograd(_bwd_t, setup_context=_setup)

__all__ = ["handle", "lgcn_propagate", "lgcn_propagate_t"]
