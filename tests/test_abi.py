"""The C-ABI library loads without a GPU, exports every symbol include/mirec.h
declares, and its host-side graph builders agree with the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import torch

from tests.conftest import LIB, ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mirec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mirec_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (mirec_\w+)", out))
    decl = declared_symbols()
    assert len(decl) >= 14
    missing = [s for s in decl if s not in exported]
    assert not missing, missing


def test_binding_covers_header():
    from furusato_recommend_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared_symbols()
    assert _lib.lib.mirec_abi_version() == 1
    assert _lib.lib.mirec_strerror(2).decode().startswith("unsupported embedding dim")


def test_struct_layout_matches():
    from furusato_recommend_amd import _lib
    sz = [ctypes.c_size_t() for _ in range(3)]
    assert _lib.lib.mirec_struct_sizes(*(ctypes.byref(x) for x in sz)) == 0
    assert [x.value for x in sz] == [ctypes.sizeof(_lib.CSR), ctypes.sizeof(_lib.Prop),
                                     ctypes.sizeof(_lib.AdamH)]


def _csr_bipartite(u, i, n_users, m_items):
    from furusato_recommend_amd._lib import lib
    u = np.ascontiguousarray(u, np.int64)
    i = np.ascontiguousarray(i, np.int64)
    n = n_users + m_items
    rowptr = np.empty(n + 1, np.int64)
    col = np.empty(2 * len(u), np.int32)
    dinv = np.empty(n, np.float32)
    rc = lib.mirec_csr_bipartite(u.ctypes.data, i.ctypes.data, len(u), n_users, m_items,
                                 rowptr.ctypes.data, col.ctypes.data, dinv.ctypes.data)
    return rc, rowptr, col, dinv


def test_csr_bipartite_matches_oracle_edge_list(golden):
    from oracle.lightgcn_oracle import degree_div, edge_index
    f = golden("lgcn_d64_L3.npz")
    nu, mi = int(f["n_users"]), int(f["m_items"])
    rc, rowptr, col, dinv = _csr_bipartite(f["train_user"], f["train_item"], nu, mi)
    assert rc == 0
    ei = edge_index(f["train_user"], f["train_item"], nu).numpy()
    # CSR by destination with stable (edge-order) rows == the reference edge list
    order = np.argsort(ei[1], kind="stable")
    assert np.array_equal(col, ei[0][order].astype(np.int32))
    assert np.array_equal(np.diff(rowptr), np.bincount(ei[1], minlength=nu + mi))
    # dinv_i * dinv_j == 1/sqrt(deg_i deg_j) of model/radj.py (r = 0.5)
    div = degree_div(torch.from_numpy(ei), nu + mi).numpy()
    w = dinv[ei[0]] * dinv[ei[1]]
    assert np.allclose(w, 1.0 / div, rtol=1e-6)
    assert dinv[nu + mi - 1] == 0.0  # the isolated item


def test_csr_rejects_out_of_range():
    rc, *_ = _csr_bipartite([0, 5], [0, 1], 3, 2)
    assert rc == 5  # MIREC_ERR_RANGE


def test_csr_from_coo_and_long_rows():
    from furusato_recommend_amd._lib import lib
    rng = np.random.default_rng(0)
    n, nnz = 50, 400
    src = rng.integers(0, n, nnz).astype(np.int64)
    dst = np.concatenate([np.zeros(100, np.int64), rng.integers(0, n, nnz - 100)])
    rowptr = np.empty(n + 1, np.int64)
    col = np.empty(nnz, np.int32)
    dinv = np.empty(n, np.float32)
    assert lib.mirec_csr_from_coo(src.ctypes.data, dst.ctypes.data, nnz, n, rowptr.ctypes.data,
                                  col.ctypes.data, dinv.ctypes.data) == 0
    order = np.argsort(dst, kind="stable")
    assert np.array_equal(col, src[order])
    deg = np.bincount(dst, minlength=n)
    assert np.allclose(dinv, np.where(deg > 0, 1 / np.sqrt(np.maximum(deg, 1)), 0))
    nl, ns = ctypes.c_int64(), ctypes.c_int64()
    split = 16
    assert lib.mirec_csr_long_rows(rowptr.ctypes.data, n, split, ctypes.byref(nl),
                                   ctypes.byref(ns), None, None, None, None) == 0
    long = np.nonzero(deg > split)[0]
    assert nl.value == len(long)
    assert ns.value == int(np.sum((deg[long] + split - 1) // split))
    lr = np.empty(nl.value, np.int32)
    lsp = np.empty(nl.value + 1, np.int64)
    sr = np.empty(ns.value, np.int32)
    sb = np.empty(ns.value, np.int64)
    assert lib.mirec_csr_long_rows(rowptr.ctypes.data, n, split, ctypes.byref(nl),
                                   ctypes.byref(ns), lr.ctypes.data, lsp.ctypes.data,
                                   sr.ctypes.data, sb.ctypes.data) == 0
    assert np.array_equal(lr, long)
    for k, r in enumerate(lr):  # segments tile each long row exactly
        segs = sb[lsp[k]:lsp[k + 1]]
        assert np.all(sr[lsp[k]:lsp[k + 1]] == r)
        assert segs[0] == rowptr[r] and np.all(np.diff(segs) == split)
        assert segs[-1] < rowptr[r + 1] <= segs[-1] + split


def test_no_kernel_reads_high_dword_through_op_sel():
    """The gfx950 code of every kernel in the library is free of packed-f32
    ops whose op_sel makes the low lane read a pair's high dword — the
    instruction shape behind the fused dX + LayerNorm-backward kernel's wrong
    upper-lane rows (tools/op_sel_repro.hip reproduces it).
    Disassembles the built library with the ROCm llvm tools, no GPU."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_scan
    ks = isa_scan.kernels(LIB)
    assert sum(1 for v in ks.values() if v["mfma"]) >= 20  # the scan sees the MFMA kernels
    assert isa_scan.hazards(LIB) == []
    # MFMA work of ANY wave on the SIMD triggers it, so no kernel at all may
    # carry such reads: any of them can run beside an MFMA kernel (the
    # public LGConv operator next to torch's GEMMs on another stream, two
    # ranks sharing a GPU).  The kernels that would otherwise get them are
    # built with MIREC_NO_PK_F32.
    others = sorted(fn for fn, v in ks.items() if v["opsel_hi"])
    assert others == [], others
