"""LGConv — drop-in for ``torch_geometric.nn.conv.LGConv`` (PyG, version
unpinned by the reference) as called at model/lgcn.py:66,82:

    y = LGConv()(x, edge_index)        # y_i = Σ_{(j→i)} x_j / sqrt(deg_i deg_j)

on any graph (not only the user–item bipartite one), with PyG's semantics:
flow source_to_target, degree = in-degree at the target with multi-edges
counted, isolated nodes give 0, ``normalize=False`` is the plain neighbour
sum.  Differentiable: the backward x̄ = Âᵀ ȳ is the same HIP SpMM on the
transposed CSR (the same CSR when the edge multiset is symmetric).  The call
goes through the registered operator ``torch.ops.mirec.lgcn_propagate``
(ops.py).

The CSR (and its transpose) is built once per ``edge_index`` and cached on
the module, keyed by the tensor's storage, shape and version; ``x`` may
have any feature width: widths outside {4, 8, ..., 256} are zero-padded to
the next supported width, widths above 256 are processed in 256-column
blocks.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .engine import propagate
from .graph import Graph


def _width(d: int) -> int:
    for w in _lib.SUPPORTED_DIMS:
        if w >= d:
            return w
    return 256


def _spmm(graph: Graph, x: torch.Tensor) -> torch.Tensor:
    n, d = x.shape
    if d in _lib.SUPPORTED_DIMS:
        xc = x.contiguous()
        y = torch.empty_like(xc)
        propagate(graph, xc, y)
        return y
    outs = []
    for c0 in range(0, d, 256):
        xb = x[:, c0:c0 + 256]
        w = _width(xb.shape[1])
        xp = F.pad(xb, (0, w - xb.shape[1])).contiguous()
        yp = torch.empty_like(xp)
        propagate(graph, xp, yp)
        outs.append(yp[:, :xb.shape[1]])
    return torch.cat(outs, 1) if len(outs) > 1 else outs[0].contiguous()


class _LGConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, graph: Graph):
        ctx.graph = graph
        return _spmm(graph, x)

    @staticmethod
    def backward(ctx, ybar):
        g = ctx.graph
        return _spmm(g if g.symmetric else g.transpose, ybar), None


class LGConv(nn.Module):
    def __init__(self, normalize: bool = True, split: int | None = None):
        super().__init__()
        self.normalize = bool(normalize)
        self.split = split
        self._key = None
        self._graph = None

    def graph_for(self, edge_index: torch.Tensor, n_nodes: int, device) -> Graph:
        key = (edge_index.data_ptr(), tuple(edge_index.shape), edge_index._version,
               int(n_nodes), str(device))
        if self._key != key:
            kw = {} if self.split is None else {"split": int(self.split)}
            self._graph = Graph.from_edge_index(edge_index.detach().cpu().numpy(), int(n_nodes),
                                                device, normalize=self.normalize, **kw)
            self._key = key
        return self._graph

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor,
                edge_weight: torch.Tensor | None = None) -> torch.Tensor:
        if edge_weight is not None:
            raise NotImplementedError("LGConv: edge_weight is not supported")
        if x.device.type != "cuda":
            raise RuntimeError("LGConv (furusato_recommend_amd) runs on a HIP device only")
        if x.dim() != 2 or x.dtype != torch.float32:
            raise ValueError("LGConv: x must be a float32 [N, D] tensor")
        g = self.graph_for(edge_index, x.shape[0], x.device)
        from .ops import handle  # torch.ops.mirec.lgcn_propagate (autograd registered)
        return torch.ops.mirec.lgcn_propagate(x, handle(g))

    def __repr__(self) -> str:
        return f"LGConv(normalize={self.normalize})"
