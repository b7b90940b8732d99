"""Device-resident user–item graph (CSR + gcn_norm) for the propagation engine.

Reference: the symmetric edge list of model/lgcn.py:53-61 (users then items
offset by n_users, both directions) and PyG's gcn_norm(add_self_loops=False)
that LGConv recomputes on every call (model/lgcn.py:82; restated in-repo by
model/radj.py:28-36).  Here both are computed once: a destination-major CSR
(int64 rowptr, int32 col, rows in the reference's edge order) and
dinv = deg^-1/2, built on the host by libmirec (mirec_csr_bipartite) and
kept in HBM for the lifetime of the model.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import CSR, check, lib

# Rows longer than this are split into segments (load balance on skewed
# item popularity).  2048 neighbours x 256 B = 512 KiB of gather per segment.
DEFAULT_SPLIT = 2048


class Graph:
    """CSR of the normalised adjacency Â = D^-1/2 A D^-1/2 (A symmetric)."""

    def __init__(self, rowptr: np.ndarray, col: np.ndarray, dinv: np.ndarray,
                 n_users: int, m_items: int, device, split: int = DEFAULT_SPLIT,
                 symmetric: bool = True):
        self.n_users = int(n_users)
        self.m_items = int(m_items)
        self.n_nodes = int(rowptr.shape[0] - 1)
        self.nnz = int(col.shape[0])
        self.symmetric = symmetric
        self.device = torch.device(device)
        self.rowptr_host = rowptr
        self.col_host = col
        self.split = int(split)
        n_long, n_seg = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib.mirec_csr_long_rows(rowptr.ctypes.data, self.n_nodes, self.split,
                                      ctypes.byref(n_long), ctypes.byref(n_seg),
                                      None, None, None, None), "csr_long_rows")
        self.n_long, self.n_seg = n_long.value, n_seg.value
        long_rows = np.zeros(max(self.n_long, 1), np.int32)
        long_segptr = np.zeros(self.n_long + 1, np.int64)
        seg_row = np.zeros(max(self.n_seg, 1), np.int32)
        seg_beg = np.zeros(max(self.n_seg, 1), np.int64)
        if self.n_long:
            check(lib.mirec_csr_long_rows(rowptr.ctypes.data, self.n_nodes, self.split,
                                          ctypes.byref(n_long), ctypes.byref(n_seg),
                                          long_rows.ctypes.data, long_segptr.ctypes.data,
                                          seg_row.ctypes.data, seg_beg.ctypes.data),
                  "csr_long_rows")
        dev = self.device
        self.rowptr = torch.from_numpy(rowptr).to(dev)
        self.col = torch.from_numpy(col if col.size else np.zeros(1, np.int32)).to(dev)
        self.dinv = torch.from_numpy(dinv).to(dev)
        self.long_rows = torch.from_numpy(long_rows).to(dev)
        self.long_segptr = torch.from_numpy(long_segptr).to(dev)
        self.seg_row = torch.from_numpy(seg_row).to(dev)
        self.seg_beg = torch.from_numpy(seg_beg).to(dev)
        self.csr = CSR(rowptr=self.rowptr.data_ptr(), col=self.col.data_ptr(),
                       dinv=self.dinv.data_ptr(), n_rows=self.n_nodes, nnz=self.nnz,
                       split=self.split, _pad=0, n_long=self.n_long, n_seg=self.n_seg,
                       long_rows=self.long_rows.data_ptr(),
                       long_segptr=self.long_segptr.data_ptr(),
                       seg_row=self.seg_row.data_ptr(), seg_beg=self.seg_beg.data_ptr(),
                       col_sorted=None, n_sorted=0)
        self.transpose = None  # set for non-symmetric graphs (from_edge_index)
        self.col_sorted = None
        self.pos_cdf = None  # weighted positives (set_positive_probs)
        if self.n_users > 0 and self.m_items > 0:
            self._sort_user_rows()

    def _sort_user_rows(self):
        """A sorted copy of the user rows (the positives of every user) for the
        samplers' binary-search membership test (negative_sample.py:121-126)."""
        nu = self.n_users
        n = int(self.rowptr_host[nu] - self.rowptr_host[0])
        cs = np.empty(max(n, 1), np.int32)
        check(lib.mirec_csr_sort_rows(self.rowptr_host.ctypes.data, self.col_host.ctypes.data,
                                      nu, cs.ctypes.data), "csr_sort_rows")
        self.col_sorted = torch.from_numpy(cs).to(self.device)
        self.csr.col_sorted = self.col_sorted.data_ptr()
        self.csr.n_sorted = nu

    # ------------------------------------------------------------------ build
    @classmethod
    def from_interactions(cls, train_user, train_item, n_users: int, m_items: int,
                          device, split: int = DEFAULT_SPLIT) -> "Graph":
        """trainUser / trainItem arrays (dataloader.py:93-124) → symmetric CSR."""
        u = np.ascontiguousarray(np.asarray(train_user, dtype=np.int64))
        i = np.ascontiguousarray(np.asarray(train_item, dtype=np.int64))
        if u.shape != i.shape:
            raise ValueError("train_user and train_item must have the same length")
        n = int(n_users) + int(m_items)
        rowptr = np.empty(n + 1, np.int64)
        col = np.empty(2 * u.shape[0], np.int32)
        dinv = np.empty(n, np.float32)
        check(lib.mirec_csr_bipartite(u.ctypes.data, i.ctypes.data, u.shape[0], int(n_users),
                                      int(m_items), rowptr.ctypes.data, col.ctypes.data,
                                      dinv.ctypes.data), "csr_bipartite")
        return cls(rowptr, col, dinv, n_users, m_items, device, split)

    @classmethod
    def from_edge_index(cls, edge_index, n_nodes: int, device,
                        split: int = DEFAULT_SPLIT, normalize: bool = True) -> "Graph":
        """Generic LGConv graph: edge_index[0] = source, [1] = target (PyG
        flow source_to_target; degree = in-degree at the target, multi-edges
        counted).  ``normalize=False``: plain neighbour sum (dinv = 1)."""
        ei = np.ascontiguousarray(np.asarray(edge_index, dtype=np.int64))
        src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
        nnz = src.shape[0]
        rowptr = np.empty(n_nodes + 1, np.int64)
        col = np.empty(nnz, np.int32)
        dinv = np.empty(n_nodes, np.float32)
        check(lib.mirec_csr_from_coo(src.ctypes.data, dst.ctypes.data, nnz, n_nodes,
                                     rowptr.ctypes.data, col.ctypes.data, dinv.ctypes.data),
              "csr_from_coo")
        if not normalize:
            dinv[:] = 1.0
        # Is the edge multiset symmetric?  Then Âᵀ = Â (same CSR for backward).
        fwd = np.sort(src * n_nodes + dst)
        bwd = np.sort(dst * n_nodes + src)
        symmetric = bool(np.array_equal(fwd, bwd))
        g = cls(rowptr, col, dinv, n_nodes, 0, device, split, symmetric=symmetric)
        if not symmetric:
            # Backward of y = Â x is x̄ = Âᵀ ȳ: CSR by source, same dinv.
            rowptr_t = np.empty(n_nodes + 1, np.int64)
            col_t = np.empty(nnz, np.int32)
            check(lib.mirec_csr_from_coo(dst.ctypes.data, src.ctypes.data, nnz, n_nodes,
                                         rowptr_t.ctypes.data, col_t.ctypes.data, None),
                  "csr_from_coo(transpose)")
            g.transpose = cls(rowptr_t, col_t, dinv, n_nodes, 0, device, split)
        return g

    def set_positive_probs(self, probs) -> None:
        """Per-user positive probabilities for the samplers (the sample_pow
        option of negative_sample.py:22-56: ``probs[u]`` is the probability
        vector over ``allPos[u]``, which is this CSR's user-row order).
        ``probs``: a sequence of per-user arrays, or one flat float array of
        the user rows' entries; ``None`` restores the uniform positive.  The
        row CDFs are built on the host (mirec_pos_cdf_build) and kept in HBM;
        every sampler call on this graph then draws its positive from them."""
        if probs is None:
            self.pos_cdf = None
            return
        nu = self.n_users
        n = int(self.rowptr_host[nu] - self.rowptr_host[0])
        if isinstance(probs, np.ndarray) and probs.ndim == 1:
            flat = np.ascontiguousarray(probs, dtype=np.float64)
        else:
            if len(probs) != nu:
                raise ValueError(f"probs: one array per user ({nu}), got {len(probs)}")
            deg = np.diff(self.rowptr_host[: nu + 1])
            parts = [np.asarray(p, dtype=np.float64).reshape(-1) for p in probs]
            bad = [u for u, (p, d) in enumerate(zip(parts, deg)) if p.size != d]
            if bad:
                raise ValueError(f"probs[{bad[0]}] has {parts[bad[0]].size} entries, "
                                 f"the user has {deg[bad[0]]} positives")
            flat = np.concatenate(parts) if parts else np.zeros(0)
        if flat.size != n:
            raise ValueError(f"probs: {flat.size} entries for {n} user-row entries")
        cdf = np.empty(max(n, 1), np.float64)
        check(lib.mirec_pos_cdf_build(self.rowptr_host.ctypes.data, nu, flat.ctypes.data,
                                      cdf.ctypes.data), "pos_cdf_build")
        self.pos_cdf = torch.from_numpy(cdf).to(self.device)

    # ---------------------------------------------------------------- helpers
    def degree(self) -> np.ndarray:
        return np.diff(self.rowptr_host)

    def csr_ptr(self):
        return ctypes.byref(self.csr)

    def partial_buffer(self, dim: int) -> torch.Tensor | None:
        if self.n_seg == 0:
            return None
        key = ("partial", dim)
        buf = getattr(self, "_bufs", {}).get(key)
        if buf is None:
            buf = torch.empty(self.n_seg, dim, dtype=torch.float32, device=self.device)
            self._bufs = getattr(self, "_bufs", {})
            self._bufs[key] = buf
        return buf

    def bytes_per_layer(self, dim: int, fused_acc: bool = True) -> int:
        """Algorithmic HBM bytes of one propagation layer."""
        n, nnz = self.n_nodes, self.nnz
        b = nnz * dim * 4 + nnz * 4 + (n + 1) * 8 + n * 4 + n * dim * 4
        if fused_acc:
            b += 2 * n * dim * 4
        return b


def positive_probs(config: dict):
    """The per-user positive probabilities a model config asks for: the
    reference's ``sample_pow`` (parse.py:48; negative_sample.py:22-38 loads
    ``data/sample_prob/sample_prob_<pow>.pkl``, a list of per-user arrays over
    allPos[u]) comes here as ``config["sample_probs"]`` — the arrays
    themselves (this package does not unpickle files).  None = uniform."""
    probs = config.get("sample_probs")
    if probs is None and float(config.get("sample_pow", 0) or 0) != 0:
        raise ValueError("sample_pow != 0: pass the per-user probabilities as "
                         "config['sample_probs'] (the arrays of sample_prob_*.pkl)")
    return probs


_ = _lib  # keep the module import explicit for readers
