"""SASRec (model/sasrec.py:54-502) — the self-attention block on MFMA.

In scope: the per-layer block of sasrec.py:385-397
(pre-LN → causal multi-head self-attention → dropout → residual + ReLU →
LN → Linear → dropout → residual), the masked mean pool over the first
`length` positions (:399-413), the item MLP tower (:415-421), the BPR loss
with the reference's embedding-norm term (:423-435) and OneEpoch (:437-474).
The attention core softmax(QKᵀ/√d_h + causal)·V and its backward are one
HIP launch each (csrc/attention.hip, f32 MFMA); the Linear layers run on
f32 MFMA GEMMs (csrc/gemm.hip; the QKV forward on hipBLASLt), the dropout /
residual / ReLU / LayerNorm tail of each stage is one fused row kernel
(csrc/resnorm.hip), and pooling, packing and the loss have kernels of their
own (csrc/pool.hip).  On one GPU the whole training step is replayed from a
captured HIP graph (_CapturedStep).
Out of scope: the proprietary text / feature towers of the initial item
embedding (:82-209): items start from an id embedding (N(0, 1), :205).
The reference hard-codes 8 heads (:211); `heads` is a parameter here
(BASELINE config C4 uses 2).
"""
from __future__ import annotations

import ctypes
import os
from typing import NamedTuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import linear as linear_mod
from ._lib import check, lib
from .engine import AdamGroup, AdamState, _note_raw_write
from .linear import Linear, blas_backend, linear, linear_relu
from .rows import gather_rows, gather_rows_norm


# Optional per-launch timing (tools/bench_sasrec.py): a list receiving
# (kind, start_event, end_event, (B, T, heads, head_dim), offsets or None,
# launches between the events); packed launches have T = -1 and their int32
# offsets.  ATTN_REPEAT = R > 1 times R back-to-back launches of the same
# kernel on the same operands after one untimed launch, so the interval holds
# kernel time only — in a host-bound eager step the GPU can idle between the
# start event and the launch (timing only: a backward launched R times
# leaves R times its accumulated input gradient).
ATTN_EVENTS = None
ATTN_REPEAT = 1


def _timed(kind, shape, launch, offsets=None):
    ev = ATTN_EVENTS
    if ev is None:
        return launch()
    reps = max(1, int(ATTN_REPEAT))
    if reps > 1:
        launch()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        r = launch()
    e.record()
    ev.append((kind, s, e, shape, offsets, reps))
    return r


# Attention core implementation: "wave" (csrc/attn_wave.hip, one wave per
# (sequence, head), head_dim 16 / 32 / 64), "block" (csrc/attention.hip, one
# workgroup per (sequence, head): any head_dim <= 64, length buckets) or
# "hybrid" (default): the wave forward and the workgroup backward, both on
# the longest-first sequence order.  At C4 (tools/attn_bench.py, 57 K
# tokens): forward wave 31 us / workgroup 38; backward wave (two passes)
# 95 us / workgroup 77.
ATTN_IMPL = "hybrid"


def _use_wave(dh: int) -> bool:
    return ATTN_IMPL in ("wave", "hybrid") and bool(lib.mirec_attention_wave_supported(dh))


_ORDER_CACHE: dict = {}


def _length_order(offsets, B):
    """[order (B, padded to 4) | packs (4 + 8B)] of a packed batch
    (mirec_attention_length_order), computed once per offsets tensor: every
    layer of a step shares it (a captured step launches the ordering pass
    once).  The packs start 16-byte aligned (``packs_of``)."""
    key = id(offsets)
    hit = _ORDER_CACHE.get(key)
    if hit is not None and hit[0]() is offsets and hit[1] == offsets._version:
        return hit[2]
    bp = -(-B // 4) * 4
    order = torch.empty(bp + 4 + 8 * B, dtype=torch.int32, device=offsets.device)
    check(lib.mirec_attention_length_order(offsets.data_ptr(), B, order.data_ptr(),
                                           order[bp:].data_ptr(), None, 0, 0,
                                           _lib.stream_handle()), "attention_length_order")
    import weakref
    for k in [k for k, v in _ORDER_CACHE.items() if v[0]() is None]:
        del _ORDER_CACHE[k]
    _ORDER_CACHE[key] = (weakref.ref(offsets), offsets._version, order)
    return order


def _wave_fwd(qkv, offsets, B, T, heads, dh, out, padded=False):
    """mirec_attention_wave_fwd; returns (lse [n_rows, heads], order): packed
    sequences run longest first (mirec_attention_length_order, shared by the
    layers of a step); with ``padded`` the kernel's spare workgroups zero
    out's capacity-padding rows."""
    lse = torch.empty(qkv.shape[0] if offsets is not None else B * T, heads, dtype=qkv.dtype,
                      device=qkv.device)
    order = None
    if offsets is not None and B > 0:
        order = _length_order(offsets, B)
    elif padded:
        _zero_tail(out, offsets)
    n_rows = out.shape[0] if (padded and order is not None) else 0
    _timed("fwd", (B, T if offsets is None else -1, heads, dh), lambda: check(
        lib.mirec_attention_wave_fwd(qkv.data_ptr(), _ptr(offsets), _ptr(order), B, T, heads, dh,
                                     out.data_ptr(), lse.data_ptr(), n_rows,
                                     _lib.stream_handle()),
        "attention_wave_fwd"), offsets)
    return lse, order


def _wave_bwd(qkv, out, lse, order, dout, offsets, B, T, heads, dh, dqkv):
    delta = torch.empty_like(lse)
    _timed("bwd", (B, T if offsets is None else -1, heads, dh), lambda: check(
        lib.mirec_attention_wave_bwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(),
                                     dout.data_ptr(), _ptr(offsets), _ptr(order), B, T, heads,
                                     dh, dqkv.data_ptr(), delta.data_ptr(),
                                     _lib.stream_handle()),
        "attention_wave_bwd"), offsets)


class _CausalAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads: int):
        B, T, d3 = qkv.shape
        d = d3 // 3
        dh = d // heads
        qkv = qkv.contiguous()
        out = torch.empty(B, T, d, dtype=qkv.dtype, device=qkv.device)
        ctx.heads = heads
        if _use_wave(dh):
            lse, _ = _wave_fwd(qkv, None, B, T, heads, dh, out)
            ctx.save_for_backward(qkv, out, lse)
            return out
        _timed("fwd", (B, T, heads, dh), lambda: check(lib.mirec_attention_fwd(
            qkv.data_ptr(), B, T, heads, dh, out.data_ptr(), _lib.stream_handle()),
            "attention_fwd"))
        ctx.save_for_backward(qkv)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv = ctx.saved_tensors[0]
        B, T, d3 = qkv.shape
        dh = d3 // 3 // ctx.heads
        dqkv = torch.empty_like(qkv)
        dout = dout.contiguous()
        if len(ctx.saved_tensors) == 3:
            _, out, lse = ctx.saved_tensors
            _wave_bwd(qkv, out, lse, None, dout, None, B, T, ctx.heads, dh, dqkv)
            return dqkv, None
        _timed("bwd", (B, T, ctx.heads, dh), lambda: check(lib.mirec_attention_bwd(
            qkv.data_ptr(), dout.data_ptr(), B, T, ctx.heads, dh, dqkv.data_ptr(),
            _lib.stream_handle()), "attention_bwd"))
        return dqkv, None


class Packing(NamedTuple):
    """Packed sequences: int32 ``offsets`` [B+1] on the device (sequence b =
    rows offsets[b] .. offsets[b+1]-1) and, when the sequences are ordered by
    length bucket, the host counts ``bucket_end`` (sequences [bucket_end[k-1],
    bucket_end[k]) have at most 16(k+1) positions; mirec_attention_bucketed_*)."""
    offsets: torch.Tensor
    bucket_end: tuple | None = None
    padded: bool = False  # rows past offsets[B] belong to no sequence (capacity padding)
    order: torch.Tensor | None = None  # caller position of each packed sequence (None: same)


class _CausalAttentionVarlen(torch.autograd.Function):
    """Packed sequences: qkv [n_tok, 3d], sequence b = rows offsets[b] ..
    offsets[b+1]-1 (mirec_attention_wave_*; or, with ATTN_IMPL "block",
    mirec_attention_varlen_* / mirec_attention_bucketed_* given the length
    buckets)."""

    @staticmethod
    def forward(ctx, qkv, offsets, heads: int, bucket_end=None, padded: bool = False):
        n, d3 = qkv.shape
        d = d3 // 3
        dh = d // heads
        B = offsets.numel() - 1
        qkv = qkv.contiguous()
        out = torch.empty(n, d, dtype=qkv.dtype, device=qkv.device)
        ctx.heads = heads
        ctx.bucket_end = bucket_end
        ctx.padded = padded
        # rows outside every sequence (capacity padding) are not written by
        # the attention kernels: zeroed by the ordering pass or here
        if _use_wave(dh):
            lse, order = _wave_fwd(qkv, offsets, B, 0, heads, dh, out, padded)
            ctx.save_for_backward(qkv, offsets, out, lse, order)
            return out
        if padded:
            _zero_tail(out, offsets)
        if bucket_end is None:
            launch = lambda: check(lib.mirec_attention_varlen_fwd(  # noqa: E731
                qkv.data_ptr(), offsets.data_ptr(), B, heads, dh, out.data_ptr(),
                _lib.stream_handle()), "attention_varlen_fwd")
        else:
            be = _bucket_array(bucket_end, B)
            launch = lambda: check(lib.mirec_attention_bucketed_fwd(  # noqa: E731
                qkv.data_ptr(), offsets.data_ptr(), be, heads, dh, out.data_ptr(),
                _lib.stream_handle()), "attention_bucketed_fwd")
        _timed("fwd", (B, -1, heads, dh), launch, offsets)
        ctx.save_for_backward(qkv, offsets)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, offsets = ctx.saved_tensors[:2]
        n, d3 = qkv.shape
        B = offsets.numel() - 1
        dh = d3 // 3 // ctx.heads
        dqkv = torch.empty_like(qkv)
        dout = dout.contiguous()
        if len(ctx.saved_tensors) == 5:
            out, lse, order = ctx.saved_tensors[2:]
            if ATTN_IMPL == "wave" or order is None:
                if ctx.padded:
                    _zero_tail(dqkv, offsets)
                _wave_bwd(qkv, out, lse, order, dout, offsets, B, 0, ctx.heads, dh, dqkv)
            else:  # sequences packed into workgroups, longest first, from the
                # forward's lse (no softmax reductions); its spare workgroups
                # zero the capacity padding rows
                _timed("bwd", (B, -1, ctx.heads, dh), lambda: check(
                    lib.mirec_attention_packed_bwd_lse(
                        qkv.data_ptr(), lse.data_ptr(), dout.data_ptr(), offsets.data_ptr(),
                        order[-(-B // 4) * 4:].data_ptr(), B, ctx.heads, dh, dqkv.data_ptr(),
                        n if ctx.padded else 0, _lib.stream_handle()),
                    "attention_packed_bwd_lse"), offsets)
            return dqkv, None, None, None, None
        if ctx.padded:
            _zero_tail(dqkv, offsets)
        if ctx.bucket_end is None:
            launch = lambda: check(lib.mirec_attention_varlen_bwd(  # noqa: E731
                qkv.data_ptr(), dout.data_ptr(), offsets.data_ptr(), B, ctx.heads, dh,
                dqkv.data_ptr(), _lib.stream_handle()), "attention_varlen_bwd")
        else:
            be = _bucket_array(ctx.bucket_end, B)
            launch = lambda: check(lib.mirec_attention_bucketed_bwd(  # noqa: E731
                qkv.data_ptr(), dout.data_ptr(), offsets.data_ptr(), be, ctx.heads, dh,
                dqkv.data_ptr(), _lib.stream_handle()), "attention_bucketed_bwd")
        _timed("bwd", (B, -1, ctx.heads, dh), launch, offsets)
        return dqkv, None, None, None, None


def _zero_tail(buf, offsets):
    """Zero the rows of buf past the last sequence (capacity padding) so
    they stay finite downstream (mirec_zero_tail_rows)."""
    check(lib.mirec_zero_tail_rows(buf.data_ptr(), offsets.data_ptr(), offsets.numel() - 1,
                                   buf.shape[0], buf.shape[1], _lib.stream_handle()),
          "zero_tail_rows")


def _bucket_array(bucket_end, batch: int):
    be = tuple(int(x) for x in bucket_end)
    if len(be) != 4 or be[3] != batch or any(b < a for a, b in zip((0,) + be, be)):
        raise ValueError(f"bucket_end {be} does not partition {batch} sequences")
    return (ctypes.c_int64 * 4)(*be)


def length_buckets(lengths) -> tuple[np.ndarray, tuple]:
    """Host lengths -> (stable order by bucket ceil(len/16) in 1..4, the
    bucket_end counts of that order)."""
    nb = np.clip((np.asarray(lengths, dtype=np.int64) + 15) // 16, 1, 4)
    order = np.argsort(nb, kind="stable")
    return order, tuple(int(x) for x in np.cumsum(np.bincount(nb - 1, minlength=4)))


def _ptr(t):
    return 0 if t is None else t.data_ptr()


class _BPRRowsLoss(torch.autograd.Function):
    """SASRec.loss as two kernels (mirec_bpr_rows_loss / _bwd): mean
    softplus(<u, ne> - <u, pe>) + coef * extra, with extra the embedding-norm
    term (a 0-d tensor) and coef = decay / B (sasrec.py:423-435 with its one
    'emb' parameter: the doubling accumulation leaves the norm itself)."""

    @staticmethod
    def forward(ctx, u, pn, extra, coef: float):
        """pn = [pe ; ne] ([2B, d]): one input, so its gradient is one tensor
        (no concatenation of the two halves' gradients in the backward)."""
        u, pn = u.contiguous(), pn.contiguous()
        B, d = u.shape
        pe, ne = pn[:B], pn[B:]
        x = torch.empty(2 * B, dtype=u.dtype, device=u.device)  # x, then scratch
        loss = torch.empty((), dtype=u.dtype, device=u.device)
        check(lib.mirec_bpr_rows_loss(u.data_ptr(), pe.data_ptr(), ne.data_ptr(), B, d,
                                      extra.data_ptr(), float(coef), x.data_ptr(),
                                      loss.data_ptr(), _lib.stream_handle()), "bpr_rows_loss")
        ctx.save_for_backward(u, pn, x)
        ctx.coef = float(coef)
        return loss

    @staticmethod
    def backward(ctx, g):
        u, pn, x = ctx.saved_tensors
        B, d = u.shape
        pe, ne = pn[:B], pn[B:]
        du, dpn = torch.empty_like(u), torch.empty_like(pn)
        dpe, dne = dpn[:B], dpn[B:]
        g_extra = torch.empty((), dtype=u.dtype, device=u.device)
        g = g.contiguous()
        check(lib.mirec_bpr_rows_loss_bwd(u.data_ptr(), pe.data_ptr(), ne.data_ptr(),
                                          x.data_ptr(), B, d, g.data_ptr(), ctx.coef,
                                          du.data_ptr(), dpe.data_ptr(), dne.data_ptr(),
                                          g_extra.data_ptr(), _lib.stream_handle()),
              "bpr_rows_loss_bwd")
        return du, dpn, g_extra, None


class _SegmentMean(torch.autograd.Function):
    """Mean of the packed rows of each sequence (mirec_segment_mean): x
    [n, d], int32 offsets [B+1], int64 seg [n] (the sequence of every row, B
    for padding), int64 length [B] (the divisor, sasrec.py:412)."""

    @staticmethod
    def forward(ctx, x, offsets, seg, length):
        x = x.contiguous()
        B, d = length.numel(), x.shape[1]
        out = torch.empty(B, d, dtype=x.dtype, device=x.device)
        check(lib.mirec_segment_mean(x.data_ptr(), offsets.data_ptr(), length.data_ptr(), B, d,
                                     out.data_ptr(), _lib.stream_handle()), "segment_mean")
        ctx.save_for_backward(seg, length)
        ctx.n = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        seg, length = ctx.saved_tensors
        g = g.contiguous()
        B, d = g.shape
        gx = torch.empty(ctx.n, d, dtype=g.dtype, device=g.device)
        check(lib.mirec_segment_mean_bwd(g.data_ptr(), seg.data_ptr(), length.data_ptr(), ctx.n,
                                         B, d, gx.data_ptr(), _lib.stream_handle()),
              "segment_mean_bwd")
        return gx, None, None, None


# Device uint64 [1] mixed into every dropout mask key while a step is being
# captured (None in eager mode): the host writes a fresh value before each
# graph replay (mirec_resnorm_*'s seed_base).
_SEED_BASE = None


def _dropout_seed(p: float) -> int:
    # host draw from torch's default CPU generator (no device sync)
    return int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0


class _ResNorm(torch.autograd.Function):
    """mirec_resnorm_fwd / _bwd on token rows [n, d]: out = act(res +
    dropout(z + bias)) and y = LayerNorm(out) (sasrec.py:385-397, the
    elementwise tail of a block stage).  Returns (out, y); y is None when
    ``norm`` is None; out is None in the pure-LayerNorm form (``res``,
    ``bias`` None, no ReLU, p = 0: out would equal z).  ``norm`` = (gamma,
    beta, eps) of an nn.LayerNorm."""

    @staticmethod
    def forward(ctx, res, z, bias, gamma, beta, relu: bool, p: float, eps: float, norm: bool,
                keep_out: bool = False):
        n, d = z.shape
        pure = res is None and bias is None and not relu and p == 0
        seed = _dropout_seed(p)
        base = _SEED_BASE if p > 0 else None
        out = None if pure else torch.empty_like(z)
        y = mean = rstd = None
        if norm:
            y = torch.empty_like(z)
            mean = torch.empty(n, dtype=z.dtype, device=z.device)
            rstd = torch.empty_like(mean)
        check(lib.mirec_resnorm_fwd(_ptr(res), z.data_ptr(), _ptr(bias), _ptr(gamma),
                                    _ptr(beta), n, d, int(relu), float(p), seed, _ptr(base),
                                    float(eps),
                                    _ptr(out), _ptr(y), _ptr(mean), _ptr(rstd),
                                    _lib.stream_handle()), "resnorm_fwd")
        ctx.save_for_backward(z if pure else out, mean, rstd, gamma)
        ctx.cfg = (relu, float(p), seed, res is not None, bias is not None, norm)
        ctx.seed_base = base
        ctx.set_materialize_grads(False)
        if pure and keep_out:
            # out = z, as a view: a later use of it (a residual) sends its
            # gradient back as g_out, added inside the backward kernel
            out = z.view_as(z)
        return out, y

    @staticmethod
    def backward(ctx, g_out, g_y):
        out, mean, rstd, gamma = ctx.saved_tensors
        relu, p, seed, has_res, has_bias, norm = ctx.cfg
        n, d = out.shape
        need = ctx.needs_input_grad
        if not norm:
            g_y = None
        g_out = None if g_out is None else g_out.contiguous()
        g_y = None if g_y is None else g_y.contiguous()
        d_res = torch.empty_like(out) if (has_res and need[0]) else None
        d_z = torch.empty_like(out) if need[1] else None
        d_bias = torch.empty(d, dtype=out.dtype, device=out.device) if (has_bias and need[2]) else None
        d_gamma = d_beta = None
        if g_y is not None and gamma is not None and need[3]:
            d_gamma = torch.empty_like(gamma)
        if g_y is not None and need[4]:
            d_beta = torch.empty(d, dtype=out.dtype, device=out.device)
        work = None
        if d_gamma is not None or d_beta is not None or d_bias is not None:
            work = torch.empty(int(lib.mirec_resnorm_work_floats(n, d)), dtype=out.dtype,
                               device=out.device)
        check(lib.mirec_resnorm_bwd(_ptr(g_y), _ptr(g_out), out.data_ptr(), _ptr(mean),
                                    _ptr(rstd), _ptr(gamma), n, d, int(relu), p, seed,
                                    _ptr(ctx.seed_base),
                                    _ptr(d_res), _ptr(d_z), _ptr(work), _ptr(d_gamma),
                                    _ptr(d_beta), _ptr(d_bias), _lib.stream_handle()),
              "resnorm_bwd")
        if norm and g_y is None:  # y unused downstream: no LayerNorm gradients
            d_gamma = torch.zeros_like(gamma) if need[3] and gamma is not None else None
            d_beta = torch.zeros(d, dtype=out.dtype, device=out.device) if need[4] else None
        return d_res, d_z, d_bias, d_gamma, d_beta, None, None, None, None, None


class _LinearResNorm(torch.autograd.Function):
    """_ResNorm of z = x Wᵀ with the GEMM and the row tail in one kernel
    (mirec_gemm_resnorm: z never written).  Backward: mirec_resnorm_bwd
    (d_res, d_z, d_bias, d_gamma, d_beta — the _ResNorm backward), then the
    Linear's dX = d_z W and dW = d_zᵀ x (mirec_gemm_nn_ex / mirec_gemm_tn).
    Returns (out, y); y is None when ``norm`` is False."""

    @staticmethod
    def forward(ctx, x, w, res, bias, gamma, beta, relu: bool, p: float, eps: float, norm: bool):
        n, k = x.shape
        d = w.shape[0]
        seed = _dropout_seed(p)
        base = _SEED_BASE if p > 0 else None
        out = torch.empty(n, d, dtype=x.dtype, device=x.device)
        y = mean = rstd = None
        if norm:
            y = torch.empty_like(out)
            mean = torch.empty(n, dtype=x.dtype, device=x.device)
            rstd = torch.empty_like(mean)
        check(lib.mirec_gemm_resnorm(x.data_ptr(), w.data_ptr(), n, k, d, _ptr(res), _ptr(bias),
                                     _ptr(gamma), _ptr(beta), int(relu), float(p), seed,
                                     _ptr(base), float(eps), out.data_ptr(), _ptr(y),
                                     _ptr(mean), _ptr(rstd), _lib.stream_handle()),
              "gemm_resnorm")
        ctx.save_for_backward(x, w, out, mean, rstd, gamma)
        ctx.cfg = (relu, float(p), seed, res is not None, bias is not None, norm)
        ctx.seed_base = base
        ctx.set_materialize_grads(False)
        return out, y

    @staticmethod
    def backward(ctx, g_out, g_y):
        x, w, out, mean, rstd, gamma = ctx.saved_tensors
        relu, p, seed, has_res, has_bias, norm = ctx.cfg
        n, d = out.shape
        k = x.shape[1]
        need = ctx.needs_input_grad
        if not norm:
            g_y = None
        g_out = None if g_out is None else g_out.contiguous()
        g_y = None if g_y is None else g_y.contiguous()
        want_z = need[0] or need[1]
        d_res = torch.empty_like(out) if (has_res and need[2]) else None
        d_z = torch.empty_like(out) if want_z else None
        d_bias = torch.empty(d, dtype=out.dtype, device=out.device) if (has_bias and need[3]) else None
        d_gamma = d_beta = None
        if g_y is not None and gamma is not None and need[4]:
            d_gamma = torch.empty_like(gamma)
        if g_y is not None and need[5]:
            d_beta = torch.empty(d, dtype=out.dtype, device=out.device)
        work = None
        if d_gamma is not None or d_beta is not None or d_bias is not None:
            work = torch.empty(int(lib.mirec_resnorm_work_floats(n, d)), dtype=out.dtype,
                               device=out.device)
        st = _lib.stream_handle()
        check(lib.mirec_resnorm_bwd(_ptr(g_y), _ptr(g_out), out.data_ptr(), _ptr(mean),
                                    _ptr(rstd), _ptr(gamma), n, d, int(relu), p, seed,
                                    _ptr(ctx.seed_base),
                                    _ptr(d_res), _ptr(d_z), _ptr(work), _ptr(d_gamma),
                                    _ptr(d_beta), _ptr(d_bias), st), "resnorm_bwd")
        if norm and g_y is None:  # y unused downstream: no LayerNorm gradients
            d_gamma = torch.zeros_like(gamma) if need[4] and gamma is not None else None
            d_beta = torch.zeros(d, dtype=out.dtype, device=out.device) if need[5] else None
        dx = dw = None
        if need[0]:
            dx = torch.empty_like(x)
            check(lib.mirec_gemm_nn_ex(d_z.data_ptr(), None, w.data_ptr(), dx.data_ptr(), None, 0,
                                       n, d, k, st), "gemm_nn_ex(dX)")
        if need[1]:
            dw = torch.empty_like(w)
            work2 = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, d, k)), dtype=w.dtype,
                                device=w.device)
            check(lib.mirec_gemm_tn(d_z.data_ptr(), x.data_ptr(), dw.data_ptr(), None, n, d, k,
                                    work2.data_ptr(), st), "gemm_tn(dW)")
        return dx, dw, d_res, d_bias, d_gamma, d_beta, None, None, None, None


# MIREC_GEMM_RESNORM=0: the GEMM and the row tail as two kernels (A/B)
FUSE_GEMM_RESNORM = os.environ.get("MIREC_GEMM_RESNORM", "1") != "0"


def linear_resnorm(x, w, res, bias=None, norm: nn.LayerNorm | None = None, relu: bool = False,
                   p: float = 0.0):
    """resnorm(res, linear(x, w), bias, norm, relu, p) — one kernel when the
    shapes are mirec_gemm_resnorm's (2-D aligned contiguous rows, d = 128,
    in width % 32), else the two-kernel composition."""
    d = w.shape[0]
    if (FUSE_GEMM_RESNORM and x.dim() == 2 and d == 128 and x.shape[1] % 32 == 0
            and w.shape[1] == x.shape[1] and linear_mod._aligned(x, w)
            and (res is None or (res.shape == (x.shape[0], d) and linear_mod._aligned(res)))
            and (bias is None or linear_mod._aligned(bias))):
        if norm is not None:
            gamma, beta, eps = norm.weight, norm.bias, norm.eps
        else:
            gamma = beta = None
            eps = 0.0
        return _LinearResNorm.apply(x, w, res, bias, gamma, beta, bool(relu), float(p),
                                    float(eps), norm is not None)
    return resnorm(res, linear(x, w), bias, norm, relu=relu, p=p)


def _qkv_grads(g_qkv, y, w_in, has_bias, st):
    """dW_in = g_qkvᵀ y and db_in = Σ g_qkv (one mirec_gemm_tn pass)."""
    n, m = g_qkv.shape
    k = y.shape[1]
    dw = torch.empty(m, k, dtype=y.dtype, device=y.device)
    db = torch.empty(m, dtype=y.dtype, device=y.device) if has_bias else None
    work = torch.empty(int(lib.mirec_gemm_tn_work_floats(n, m, k)), dtype=y.dtype,
                       device=y.device)
    check(lib.mirec_gemm_tn(g_qkv.data_ptr(), y.data_ptr(), dw.data_ptr(), _ptr(db), n, m, k,
                            work.data_ptr(), st), "gemm_tn(dW_in)")
    return dw, db


def _qkv_forward(y, w_in, b_in, st):
    """qkv = y W_inᵀ + b_in (mirec_gemm_nt)."""
    n, k = y.shape
    m = w_in.shape[0]
    qkv = torch.empty(n, m, dtype=y.dtype, device=y.device)
    check(lib.mirec_gemm_nt(y.data_ptr(), w_in.data_ptr(), _ptr(b_in), qkv.data_ptr(), n, k, m,
                            st), "gemm_nt(qkv)")
    return qkv


class _LnQkvHead(torch.autograd.Function):
    """The first layer's LayerNorm and QKV projection as one node:
    y = LN_a(x) (mirec_resnorm_fwd), qkv = y W_inᵀ + b_in (mirec_gemm_nt);
    x is also returned (a view) as the first residual, so its gradient comes
    back here.  Backward: dW_in, db_in = g_qkvᵀ y, Σ g_qkv; then g_y = g_qkv
    W_in and the LayerNorm backward (+ the residual's gradient) in one
    kernel (mirec_gemm_nn_resnorm_bwd: g_y never written).  Returns
    (x, qkv)."""

    @staticmethod
    def forward(ctx, x, g_a, b_a, w_in, b_in, eps: float):
        n, d = x.shape
        st = _lib.stream_handle()
        y = torch.empty_like(x)
        mean = torch.empty(n, dtype=x.dtype, device=x.device)
        rstd = torch.empty_like(mean)
        check(lib.mirec_resnorm_fwd(None, x.data_ptr(), None, _ptr(g_a), _ptr(b_a), n, d, 0, 0.0,
                                    0, None, float(eps), None, y.data_ptr(), mean.data_ptr(),
                                    rstd.data_ptr(), st), "resnorm_fwd(LN_a)")
        qkv = _qkv_forward(y, w_in, b_in, st)
        ctx.save_for_backward(x, y, mean, rstd, g_a, w_in)
        ctx.has_bias = b_in is not None
        ctx.set_materialize_grads(False)
        return x.view_as(x), qkv

    @staticmethod
    def backward(ctx, g_x, g_qkv):
        x, y, mean, rstd, g_a, w_in = ctx.saved_tensors
        n, d = x.shape
        st = _lib.stream_handle()
        f32 = dict(dtype=x.dtype, device=x.device)
        g_x = None if g_x is None else g_x.contiguous()
        dw_in = db_in = None
        if g_qkv is None:  # qkv unused downstream: only the residual's gradient
            return ((torch.zeros_like(x) if g_x is None else g_x),
                    torch.zeros_like(g_a) if g_a is not None else None,
                    torch.zeros(d, **f32), torch.zeros_like(w_in), None, None)
        d_ga = torch.empty_like(g_a) if g_a is not None else None
        d_ba = torch.empty(d, **f32)
        dx = torch.empty_like(x)
        if g_qkv is not None:
            g_qkv = g_qkv.contiguous()
            dw_in, db_in = _qkv_grads(g_qkv, y, w_in, ctx.has_bias, st)
            work = torch.empty(int(lib.mirec_gemm_nn_resnorm_bwd_work_floats(n, d)), **f32)
            check(lib.mirec_gemm_nn_resnorm_bwd(g_qkv.data_ptr(), w_in.data_ptr(), n,
                                                w_in.shape[0], d, _ptr(g_x), x.data_ptr(),
                                                mean.data_ptr(), rstd.data_ptr(), _ptr(g_a), 0,
                                                0.0, 0, None, dx.data_ptr(), None,
                                                work.data_ptr(), _ptr(d_ga), d_ba.data_ptr(),
                                                None, st), "gemm_nn_resnorm_bwd(LN_a)")
        return dx, d_ga, d_ba, dw_in, db_in, None


class _BlockTail(torch.autograd.Function):
    """Everything of a SASRec layer after the attention core (sasrec.py:
    390-397) as one node: h, y_f = LR(o W_oᵀ; res, b_o, LN_f, ReLU) and
    res', y' = LR(y_f W_fᵀ; h, b_f, LN_next), each forward one
    mirec_gemm_resnorm, and — when the next layer's projection is passed —
    its qkv' = y' W_inᵀ + b_in.  h and y_f (and y') are used only inside the
    node, so every input gradient of a Linear here is handed straight to the
    row tail before it in the same kernel (mirec_gemm_nn_resnorm_bwd: g_y',
    g_y_f never written): [g_y' = g_qkv' W_in -> resnorm_bwd(stage 2)] (or
    resnorm_bwd(stage 2) alone) -> dW_f, then [g_y_f = d_z2 W_f ->
    resnorm_bwd(stage 1)] -> dW_o, dO.  Returns (res', qkv' or y' or None)."""

    @staticmethod
    def forward(ctx, o, res, w_o, b_o, g_f, be_f, w_f, b_f, g_n, be_n, w_in, b_in, p: float,
                eps_f: float, eps_n: float, has_next: bool):
        n, k = o.shape
        d = w_o.shape[0]
        st = _lib.stream_handle()
        seeds, base = [], (_SEED_BASE if p > 0 else None)

        def stage(x, w, r, b, gam, bet, relu, eps, norm):
            seed = _dropout_seed(p)
            seeds.append(seed)
            out = torch.empty(n, d, dtype=x.dtype, device=x.device)
            y = mean = rstd = None
            if norm:
                y = torch.empty_like(out)
                mean = torch.empty(n, dtype=x.dtype, device=x.device)
                rstd = torch.empty_like(mean)
            check(lib.mirec_gemm_resnorm(x.data_ptr(), w.data_ptr(), n, x.shape[1], d, r.data_ptr(),
                                         _ptr(b), _ptr(gam), _ptr(bet), int(relu), float(p), seed,
                                         _ptr(base), float(eps), out.data_ptr(), _ptr(y),
                                         _ptr(mean), _ptr(rstd), st), "gemm_resnorm")
            return out, y, mean, rstd

        h, y_f, mean1, rstd1 = stage(o, w_o, res, b_o, g_f, be_f, True, eps_f, True)
        res2, y2, mean2, rstd2 = stage(y_f, w_f, h, b_f, g_n, be_n, False, eps_n, has_next)
        qkv = _qkv_forward(y2, w_in, b_in, st) if w_in is not None else None
        ctx.save_for_backward(o, w_o, h, mean1, rstd1, g_f, y_f, w_f, res2, mean2, rstd2, g_n,
                              y2 if w_in is not None else None, w_in)
        ctx.cfg = (float(p), seeds, has_next, b_o is not None, b_f is not None,
                   b_in is not None)
        ctx.seed_base = base
        ctx.set_materialize_grads(False)
        return res2, (qkv if w_in is not None else y2)

    @staticmethod
    def backward(ctx, g_res2, g_second):
        (o, w_o, h, mean1, rstd1, g_f, y_f, w_f, res2, mean2, rstd2, g_n, y2,
         w_in) = ctx.saved_tensors
        p, (seed1, seed2), has_next, has_bo, has_bf, has_bin = ctx.cfg
        n, d = h.shape
        k = o.shape[1]
        st = _lib.stream_handle()
        base = _ptr(ctx.seed_base)
        g_res2 = None if g_res2 is None else g_res2.contiguous()
        g_second = None if (g_second is None or not has_next) else g_second.contiguous()
        f32 = dict(dtype=h.dtype, device=h.device)
        # stage 2: res' = h + drop(y_f W_fᵀ + b_f), y' = LN_next(res')
        # (+ qkv' = y' W_inᵀ + b_in)
        d_h = torch.empty_like(h)
        d_z2 = torch.empty_like(h)
        d_bf = torch.empty(d, **f32) if has_bf else None
        d_gn = torch.empty(d, **f32) if (g_second is not None and g_n is not None) else None
        d_ben = torch.empty(d, **f32) if g_second is not None else None
        dw_in = db_in = None
        if w_in is not None and g_second is not None:
            dw_in, db_in = _qkv_grads(g_second, y2, w_in, has_bin, st)
            work2 = torch.empty(int(lib.mirec_gemm_nn_resnorm_bwd_work_floats(n, d)), **f32)
            check(lib.mirec_gemm_nn_resnorm_bwd(g_second.data_ptr(), w_in.data_ptr(), n,
                                                w_in.shape[0], d, _ptr(g_res2), res2.data_ptr(),
                                                mean2.data_ptr(), rstd2.data_ptr(), _ptr(g_n), 0,
                                                p, seed2, base, d_h.data_ptr(), d_z2.data_ptr(),
                                                work2.data_ptr(), _ptr(d_gn), _ptr(d_ben),
                                                _ptr(d_bf), st), "gemm_nn_resnorm_bwd(stage 2)")
        else:
            g_y2 = None if w_in is not None else g_second
            work = torch.empty(int(lib.mirec_resnorm_work_floats(n, d)), **f32)
            if g_y2 is None:
                d_gn = d_ben = None
            check(lib.mirec_resnorm_bwd(_ptr(g_y2), _ptr(g_res2), res2.data_ptr(), _ptr(mean2),
                                        _ptr(rstd2), _ptr(g_n), n, d, 0, p, seed2, base,
                                        d_h.data_ptr(), d_z2.data_ptr(), work.data_ptr(),
                                        _ptr(d_gn), _ptr(d_ben), _ptr(d_bf), st),
                  "resnorm_bwd(stage 2)")
        if has_next and d_ben is None:  # y' unused downstream: no LayerNorm gradients
            d_gn = torch.zeros_like(g_n) if g_n is not None else None
            d_ben = torch.zeros(d, **f32)
        if w_in is not None and dw_in is None:
            dw_in = torch.zeros_like(w_in)
            db_in = torch.zeros(w_in.shape[0], **f32) if has_bin else None
        dw_f = torch.empty_like(w_f)
        work_tn = torch.empty(max(int(lib.mirec_gemm_tn_work_floats(n, d, d)),
                                  int(lib.mirec_gemm_tn_work_floats(n, d, k))), **f32)
        check(lib.mirec_gemm_tn(d_z2.data_ptr(), y_f.data_ptr(), dw_f.data_ptr(), None, n, d, d,
                                work_tn.data_ptr(), st), "gemm_tn(dW_f)")
        # stage 1 from g_y_f = d_z2 W_f, in one kernel
        d_res = torch.empty_like(h)
        d_z1 = torch.empty_like(h)
        d_bo = torch.empty(d, **f32) if has_bo else None
        d_gf = torch.empty(d, **f32) if g_f is not None else None
        d_bef = torch.empty(d, **f32)
        work1 = torch.empty(int(lib.mirec_gemm_nn_resnorm_bwd_work_floats(n, d)), **f32)
        check(lib.mirec_gemm_nn_resnorm_bwd(d_z2.data_ptr(), w_f.data_ptr(), n, d, d,
                                            d_h.data_ptr(), h.data_ptr(), mean1.data_ptr(),
                                            rstd1.data_ptr(), _ptr(g_f), 1, p, seed1, base,
                                            d_res.data_ptr(), d_z1.data_ptr(), work1.data_ptr(),
                                            _ptr(d_gf), d_bef.data_ptr(), _ptr(d_bo), st),
              "gemm_nn_resnorm_bwd(stage 1)")
        dw_o = torch.empty_like(w_o)
        check(lib.mirec_gemm_tn(d_z1.data_ptr(), o.data_ptr(), dw_o.data_ptr(), None, n, d, k,
                                work_tn.data_ptr(), st), "gemm_tn(dW_o)")
        do = torch.empty_like(o)
        check(lib.mirec_gemm_nn_ex(d_z1.data_ptr(), None, w_o.data_ptr(), do.data_ptr(), None, 0,
                                   n, d, k, st), "gemm_nn_ex(dO)")
        return (do, d_res, dw_o, d_bo, d_gf, d_bef, dw_f, d_bf, d_gn, d_ben, dw_in, db_in,
                None, None, None, None)


# MIREC_BLOCK_TAIL=0: the two stages as separate linear_resnorm nodes (A/B)
FUSE_BLOCK_TAIL = os.environ.get("MIREC_BLOCK_TAIL", "1") != "0"
# MIREC_FUSE_QKV=0: the QKV projections as their own nodes after each LayerNorm (A/B)
FUSE_QKV = os.environ.get("MIREC_FUSE_QKV", "1") != "0"


def block_tail(o, res, w_o, b_o, norm_f: nn.LayerNorm, w_f, b_f,
               norm_next: nn.LayerNorm | None, p: float = 0.0, next_proj=None):
    """(res', y') of a layer after its attention core: h, y_f =
    linear_resnorm(o, W_o, res, b_o, LN_f, ReLU); res', y' =
    linear_resnorm(y_f, W_f, h, b_f, LN_next) — one autograd node with a
    fused backward when the shapes are the kernels' (d = 128, aligned
    contiguous rows), else the two nodes.  With ``next_proj`` = (W_in, b_in)
    of the next layer's attention (and norm_next) it returns (res', qkv' =
    y' W_inᵀ + b_in) instead, the projection inside the same node."""
    d = w_o.shape[0]
    al = linear_mod._aligned
    w_in, b_in = next_proj if next_proj is not None else (None, None)
    if next_proj is not None and norm_next is None:
        raise ValueError("next_proj needs norm_next (the projection reads LN_next's output)")
    if (FUSE_BLOCK_TAIL and FUSE_GEMM_RESNORM and o.dim() == 2 and d == 128
            and o.shape[1] % 32 == 0 and w_o.shape[1] == o.shape[1] and w_f.shape == (d, d)
            and res.shape == (o.shape[0], d) and al(o, w_o, w_f, res)
            and all(t is None or al(t) for t in (b_o, b_f))
            and (w_in is None or (w_in.shape[1] == d and w_in.shape[0] % 128 == 0
                                  and w_in.shape[0] % 32 == 0 and al(w_in)
                                  and (b_in is None or al(b_in))))):
        g_n = be_n = None
        eps_n = 0.0
        if norm_next is not None:
            g_n, be_n, eps_n = norm_next.weight, norm_next.bias, norm_next.eps
        return _BlockTail.apply(o, res, w_o, b_o, norm_f.weight, norm_f.bias, w_f, b_f, g_n,
                                be_n, w_in, b_in, float(p), float(norm_f.eps), float(eps_n),
                                norm_next is not None)
    h, y = linear_resnorm(o, w_o, res, b_o, norm_f, relu=True, p=p)
    res2, y2 = linear_resnorm(y, w_f, h, b_f, norm_next, p=p)
    return (res2, linear(y2, w_in, b_in)) if w_in is not None else (res2, y2)


def ln_qkv_head(x, norm: nn.LayerNorm, w_in, b_in):
    """(x, LN(x) W_inᵀ + b_in): the first layer's LayerNorm + QKV projection
    (x returned as the first residual) — one node with a fused backward
    (_LnQkvHead) when the shapes are the kernels', else resnorm + linear."""
    al = linear_mod._aligned
    d = x.shape[-1]
    if (FUSE_BLOCK_TAIL and x.dim() == 2 and d == 128 and al(x, w_in)
            and w_in.shape[1] == d and w_in.shape[0] % 128 == 0 and (b_in is None or al(b_in))):
        return _LnQkvHead.apply(x, norm.weight, norm.bias, w_in, b_in, float(norm.eps))
    res, y = resnorm(None, x, norm=norm, keep_out=True)
    return res, linear(y, w_in, b_in)


def resnorm(res, z, bias=None, norm: nn.LayerNorm | None = None, relu: bool = False,
            p: float = 0.0, keep_out: bool = False):
    """(out, y) of _ResNorm for rows of width d = z.shape[-1] (any leading
    shape); ``norm`` an nn.LayerNorm over d or None.  ``keep_out``: in the
    pure-LayerNorm form return out (= z) too, so that z's other use (the
    block's residual) is taken from it and its gradient joins this node's
    backward (no separate gradient accumulation)."""
    shape = z.shape
    d = shape[-1]
    if d % 4 or not 4 <= d <= 1024:
        raise ValueError("fused block rows need d % 4 == 0 and 4 <= d <= 1024")
    z2 = z.reshape(-1, d).contiguous()
    r2 = None if res is None else res.reshape(-1, d).contiguous()
    if norm is not None:
        gamma, beta, eps = norm.weight, norm.bias, norm.eps
    else:
        gamma = beta = None
        eps = 0.0
    out, y = _ResNorm.apply(r2, z2, bias, gamma, beta, relu, p, eps, norm is not None, keep_out)
    return (None if out is None else out.view(shape)), (None if y is None else y.view(shape))


class CausalSelfAttention(nn.Module):
    """nn.MultiheadAttention(d, heads, batch_first=True) called as
    attn(x, x, x, attn_mask=causal)[0] — same parameter names
    (in_proj_weight, in_proj_bias, out_proj.weight, out_proj.bias), so
    reference state dicts load unchanged."""

    def __init__(self, d: int, heads: int, device=None):
        super().__init__()
        if d % heads or not 1 <= d // heads <= 64:
            raise ValueError("head_dim = d / heads must be an integer <= 64")
        self.heads = heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d, device=device))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d, device=device))
        self.out_proj = Linear(d, d, device=device)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, x, offsets=None):
        """x [B, T, d] (padded), or packed [n_tok, d] with int32 ``offsets``
        [B+1] (sequence b = rows offsets[b] .. offsets[b+1]-1) or a Packing."""
        return self.out_proj(self.core(x, offsets))

    def core(self, x, offsets=None):
        """The heads' outputs before the out-projection."""
        return self.core_from_qkv(linear(x, self.in_proj_weight, self.in_proj_bias), offsets)

    def core_from_qkv(self, qkv, offsets=None):
        """core() after the QKV projection (qkv [.., 3d])."""
        if offsets is None:
            return _CausalAttention.apply(qkv, self.heads)
        if isinstance(offsets, Packing):
            return _CausalAttentionVarlen.apply(qkv, offsets.offsets, self.heads,
                                                offsets.bucket_end, offsets.padded)
        return _CausalAttentionVarlen.apply(qkv, offsets, self.heads)


class SequenceData:
    """Last <= max_len train items per user (SequenceDataset, sasrec.py:34-52)
    as a padded int32 [n_users, max_len] table + lengths (device)."""

    def __init__(self, sequences, device, max_len: int = 50):
        n = len(sequences)
        items = np.zeros((n, max_len), np.int32)
        lens = np.zeros(n, np.int64)
        for u, s in enumerate(sequences):
            s = np.asarray(s)[-max_len:]
            items[u, :len(s)] = s
            lens[u] = len(s)
        self.items = torch.from_numpy(items).to(device)
        self.length = torch.from_numpy(lens).to(device)
        self.length_host = lens
        self.max_len = max_len
        self._check()

    def _check(self):
        if self.max_len > 64:
            raise ValueError("SASRec attention supports sequences of at most 64 items")

    @classmethod
    def synthetic(cls, n_users, m_items, device, max_len=50, min_len=5, seed=0):
        g = torch.Generator().manual_seed(seed)
        lens = torch.randint(min_len, max_len + 1, (n_users,), generator=g)
        obj = cls.__new__(cls)
        items = torch.randint(0, m_items, (n_users, max_len), generator=g, dtype=torch.int32)
        items[torch.arange(max_len)[None, :] >= lens[:, None]] = 0
        obj.items, obj.length, obj.max_len = items.to(device), lens.to(device), max_len
        obj.length_host = lens.numpy()
        obj._check()
        return obj


class SASRec(nn.Module):
    def __init__(self, config: dict, dataset, sequences: SequenceData | None = None):
        super().__init__()
        self.config = config
        self.n_user = self.num_users = int(dataset.n_users)
        self.m_item = self.num_items = int(dataset.m_items)
        d = self.latent_dim = int(config.get("recdim", 128))
        L = self.num_layers = int(config.get("layer", 2))
        heads = int(config.get("heads", 8))
        self.device = torch.device(config.get("device", "cuda:0"))
        if self.device.type != "cuda":
            raise RuntimeError("SASRec (furusato_recommend_amd) runs on a HIP device only")
        dev = self.device
        self.item_id_embedding = nn.Embedding(self.m_item, d, device=dev)
        nn.init.normal_(self.item_id_embedding.weight)  # sasrec.py:205
        self.dropout = nn.Dropout(float(config.get("dropout_p", 0.2)))
        self.attn_layers = nn.ModuleList([CausalSelfAttention(d, heads, dev) for _ in range(L)])
        self.attn_norm_layers = nn.ModuleList([nn.LayerNorm(d, device=dev) for _ in range(L)])
        self.ffn_norm_layers = nn.ModuleList([nn.LayerNorm(d, device=dev) for _ in range(L)])
        self.ffn_layers = nn.ModuleList([Linear(d, d, device=dev) for _ in range(L)])
        self.item_linears = nn.ModuleList([Linear(d, d, device=dev) for _ in range(L - 1)])
        self.item_last_proj = Linear(d, d, device=dev)
        if sequences is None:
            sequences = SequenceData(dataset.allPos, dev)
        self.seq = sequences
        self.optims = AdamGroup(AdamState(p, lr=config["lr"]) for p in self.parameters())
        # the item table's gradient in the sorted form, its Adam fused with
        # forming it (graphsage.TableGrad; config "table_grad": "dense" = the
        # materialised gradient + dense Adam)
        self._table_state = next(s for s in self.optims
                                 if s.param is self.item_id_embedding.weight)
        self._rest_optims = AdamGroup(s for s in self.optims if s is not self._table_state)
        self._tg = None
        mode = config.get("table_grad", "sorted")
        if mode not in ("sorted", "atomic", "dense"):
            raise ValueError(f"table_grad: sorted | atomic | dense, not {mode!r}")
        if mode != "dense":
            from .graphsage import TableGrad
            self._tg = TableGrad(self.m_item, 0, d, dev)
            self._tg.atomic = mode == "atomic"
        # the table's norm after the last fused Adam ([1] of the kernel's two
        # slice norms; the one-slice table is slice 1) and the table state it
        # belongs to: the next forward reads it instead of a pass over the table
        self._norm_buf = torch.zeros(2, device=dev)
        self._norm_tok = None

    # ------------------------------------------------------------- blocks
    def oneblock(self, x, layer, offsets=None):
        """sasrec.py:385-397 (padded [B, T, d], or packed [n_tok, d] with
        ``offsets``: every other op of the block is per position)."""
        init_x = x
        x = self.attn_norm_layers[layer](x)
        x = self.attn_layers[layer](x, offsets)
        x = self.dropout(x)
        x = (init_x + x).relu()
        init_x = x
        x = self.ffn_norm_layers[layer](x)
        x = self.ffn_layers[layer](x)
        return init_x + self.dropout(x)

    def blocks(self, x, offsets=None):
        """Every layer's oneblock, with the elementwise tail of each stage in
        one fused row pass (mirec_resnorm_*: dropout + residual (+ ReLU) +
        the next LayerNorm, the linear biases folded in).  Same values as
        the oneblock chain (dropout draws differ: counter hash)."""
        if not self.config.get("fused_rows", True):  # A/B: the torch composition
            for i in range(self.num_layers):
                x = self.oneblock(x, i, offsets)
            return x
        p = self.dropout.p if self.training else 0.0
        L = self.num_layers
        if FUSE_QKV and x.dim() == 2:
            # every LayerNorm -> QKV projection pair inside one node (the head
            # node, then each layer tail with the next layer's projection):
            # the projection's input gradient meets the LayerNorm backward
            # in one kernel
            a0 = self.attn_layers[0]
            res, qkv = ln_qkv_head(x, self.attn_norm_layers[0], a0.in_proj_weight,
                                   a0.in_proj_bias)
            for i in range(L):
                attn, ffn = self.attn_layers[i], self.ffn_layers[i]
                o = attn.core_from_qkv(qkv, offsets)
                last = i + 1 == L
                nxt = None if last else self.attn_norm_layers[i + 1]
                proj = None if last else (self.attn_layers[i + 1].in_proj_weight,
                                          self.attn_layers[i + 1].in_proj_bias)
                res, qkv = block_tail(o, res, attn.out_proj.weight, attn.out_proj.bias,
                                      self.ffn_norm_layers[i], ffn.weight, ffn.bias, nxt, p=p,
                                      next_proj=proj)
            return res
        # the first residual is taken from the LayerNorm node (keep_out): its
        # gradient and the LayerNorm's meet inside one backward kernel
        res, y = resnorm(None, x, norm=self.attn_norm_layers[0], keep_out=True)
        for i in range(L):
            attn = self.attn_layers[i]
            # out-projection / FFN Linear and each stage's row tail in one
            # kernel (the biases ride in the row tails), both stages one
            # autograd node with a fused backward
            ffn = self.ffn_layers[i]
            nxt = self.attn_norm_layers[i + 1] if i + 1 < L else None
            res, y = block_tail(attn.core(y, offsets), res, attn.out_proj.weight,
                                attn.out_proj.bias, self.ffn_norm_layers[i], ffn.weight,
                                ffn.bias, nxt, p=p)
        return res

    def forward_user(self, x, length):
        """sasrec.py:399-413: blocks, then the mean over the first `length`
        positions of each sequence."""
        x = self.blocks(x)
        T = x.shape[1]
        mask = (torch.arange(T, device=x.device)[None, :] < length[:, None]).to(x.dtype)
        return (x * mask.unsqueeze(2)).sum(1) / length.to(x.dtype).unsqueeze(1)

    def forward_user_packed(self, x, offsets, seg, length):
        """forward_user on packed sequences: x [n_tok, d], ``seg`` [n_tok]
        the packed sequence of every row (B for capacity padding rows, which
        the pool drops), ``length`` [B] in packed order.  Padding positions never reach a real position under
        the causal mask and are excluded from the pool, so this equals
        forward_user on the padded batch while skipping them."""
        x = self.blocks(x, offsets)
        packed = isinstance(offsets, Packing)
        pooled = _SegmentMean.apply(x, offsets.offsets if packed else offsets, seg, length)
        if packed and offsets.order is not None:  # back to the caller's order
            pooled = torch.empty_like(pooled).index_copy(0, offsets.order, pooled)
        return pooled

    def packed_input(self, users):
        """(x [n_tok, d], packing, seg [n_tok], length [B]) of the users'
        sequences.  The token count is taken from the host copy of the
        lengths (host ``users``: no device synchronisation)."""
        ids, packing, seg, length = self.packed_ids(users)
        return gather_rows(self.item_id_embedding.weight, ids), packing, seg, length

    def packed_ids(self, users):
        """packed_input's item ids [n_tok] (int32) instead of their rows.

        With config "attn_buckets" the sequences are packed in length-bucket
        order (ceil(len/16) = 1..4, stable), so each bucket's attention runs
        on a workgroup sized for it (Packing.bucket_end, Packing.order = the
        user position of every packed sequence); ``seg`` (the packed sequence
        of every row) and ``length`` follow the packed order, and
        forward_user_packed returns the users in the caller's order."""
        if torch.is_tensor(users) and users.is_cuda:
            u_host = users.cpu().numpy()
        else:
            u_host = np.asarray(users)
        B = len(u_host)
        lens_h = self.seq.length_host[u_host]
        n_tok = int(lens_h.sum())
        dev = self.device
        if self.config.get("attn_buckets", False):
            order, bucket_end = length_buckets(lens_h)
            up = self._upload(np.concatenate([u_host, order]))
            perm = up[B:]
            u_p = up[:B][perm]
        else:  # default: one 64-row bucket, users in the caller's order
            bucket_end = perm = None
            u_p = self._upload(u_host)
        length_p = self.seq.length[u_p]
        offsets = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        offsets[1:] = torch.cumsum(length_p, 0).to(torch.int32)
        seg = torch.repeat_interleave(torch.arange(B, device=dev), length_p, output_size=n_tok)
        pos = torch.arange(n_tok, device=dev) - offsets[seg].long()
        ids = self.seq.items[u_p[seg], pos]
        return ids, Packing(offsets, bucket_end, False, perm), seg, length_p

    def _upload(self, host_ids) -> torch.Tensor:
        """int64 host ids -> device without a stream sync: a pageable H2D copy
        blocks until the stream drains, so the ids go through one of two
        pinned staging buffers (each reused only after its previous copy's
        event completed)."""
        n = len(host_ids)
        st = getattr(self, "_stage", None)
        if st is None or st[0][0].numel() < n:
            st = ([torch.empty(max(n, 4096), dtype=torch.int64).pin_memory() for _ in range(2)],
                  [None, None], [0])
            self._stage = st
        bufs, events, turn = st
        k = turn[0]
        turn[0] ^= 1
        if events[k] is not None:
            events[k].synchronize()
        buf = bufs[k][:n]
        buf.numpy()[:] = np.asarray(host_ids, dtype=np.int64)
        out = buf.to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        events[k] = ev
        return out

    @torch.no_grad()
    def sample_pairs(self, users: torch.Tensor, seed: int, offset: int = 0):
        """Device (positive, negative) item ids [2, B] (int64) for device user
        ids: a uniform element of each user's sequence and a uniform item
        (mirec_seq_sample, one launch)."""
        users = users.to(device=self.device, dtype=torch.int64).contiguous()
        items, length = self.seq.items.contiguous(), self.seq.length.contiguous()
        if items.dtype != torch.int32 or length.dtype != torch.int64:
            raise ValueError("SequenceData: int32 items and int64 lengths expected")
        out = torch.empty(2, users.numel(), dtype=torch.int64, device=self.device)
        check(lib.mirec_seq_sample(users.data_ptr(), users.numel(), items.data_ptr(),
                                   items.shape[1], length.data_ptr(), self.m_item,
                                   ctypes.c_uint64(seed), ctypes.c_uint64(offset),
                                   out.data_ptr(), _lib.stream_handle()), "seq_sample")
        return out

    def forward_item(self, x):
        """sasrec.py:415-421."""
        for lin in self.item_linears:
            x = linear_relu(x, lin.weight, lin.bias)
        return self.item_last_proj(x)

    def sequence_input(self, users):
        """Padded item-embedding sequences [B, T, d] (zero past `length`,
        pad_sequence in OneEpoch, sasrec.py:449-455) and lengths.  The lookup
        is one row gather whose backward scatter-adds into the table."""
        items = self.seq.items[users.long()]
        length = self.seq.length[users.long()]
        T = self.seq.max_len
        mask = (torch.arange(T, device=items.device)[None, :] < length[:, None])
        ids = torch.where(mask, items, torch.full_like(items, -1))
        return gather_rows(self.item_id_embedding.weight, ids), length

    def loss(self, user_emb, pos_emb, neg_emb):
        """sasrec.py:423-435 (norm of every 'emb' parameter, accumulated by
        doubling as in the reference)."""
        pos_scores = torch.sum(user_emb * pos_emb, dim=1)
        neg_scores = torch.sum(user_emb * neg_emb, dim=1)
        all_param = 0
        for k, v in self.named_parameters():
            if "emb" in k:
                all_param = all_param + all_param + v.norm(2)
        all_param = all_param / user_emb.size(0)
        loss = torch.mean(F.softplus(neg_scores - pos_scores))
        return loss + all_param * self.config["decay"]

    # DenseGradDataParallel passes table_by_hook: the captured step can be
    # split around its gradient exchange
    captures_dp_step = True

    def stageOne(self, users, pos, neg, grad_hook=None, loss_scale: float = 1.0,
                 table_by_hook: bool | None = None):
        """One BPR step on packed sequences.  ``loss_scale`` scales the
        gradient (1/world_size under data parallelism); ``grad_hook`` runs
        between backward and Adam (DenseGradDataParallel's all-reduce).
        With config "graph" (default on) the step replays a captured HIP graph
        (_CapturedStep): the whole step for a single process; under data
        parallelism (a hook and ``table_by_hook`` — whether the hook itself
        steps the item table — given) two graphs, the packing / forward /
        loss / backward one and the Adam one, with the hook's collectives
        run between the two replays.  Otherwise the step runs eagerly.  The
        projections run on the BLAS backend of config "blas" (default:
        hipBLASLt in the captured step, where its faster kernels win;
        rocBLAS in the eager step, which is host-bound and rocBLAS launches
        cost less host time)."""
        if self.config.get("graph", True) and len(users) > 0:
            if grad_hook is None and loss_scale == 1.0:
                return self._graph_step(users, pos, neg)
            if grad_hook is not None and table_by_hook is not None:
                return self._graph_step(users, pos, neg, grad_hook, float(loss_scale),
                                        bool(table_by_hook))
        with blas_backend(self.config.get("blas", "cublas")):
            return self._stage_one(users, pos, neg, grad_hook, loss_scale)

    def graph_blas(self) -> str:
        return self.config.get("blas", "cublaslt")

    def _stage_one(self, users, pos, neg, grad_hook, loss_scale):
        for p in self.parameters():
            p.grad = None
        pos, neg = (torch.as_tensor(t).to(self.device) for t in (pos, neg))
        ids, packing, seg, length = self.packed_ids(users)
        loss = self._step_body(ids, packing, seg, length, pos, neg, loss_scale)
        if grad_hook is not None:
            tg = self._tg
            if (tg is not None and tg.pending and self.item_id_embedding.weight.grad is None
                    and not getattr(self, "_tg_routed", False)):
                # the hook (an all-reduce, a test) sees every gradient
                self.item_id_embedding.weight.grad = tg.materialize(
                    self.item_id_embedding.weight.detach())
            grad_hook()
        self.optimizer_step()
        return loss.detach()

    @torch.no_grad()
    def optimizer_step(self, h_dev: torch.Tensor | None = None):
        """Adam over every parameter (sasrec.py:468-471): the item table
        through the fused kernel from the pending sorted gradient, the rest
        with the multi-tensor kernel; or all of them densely when the
        table's gradient was materialised.  ``h_dev``: device hyper-parameters
        (captured step)."""
        tg = self._tg
        w = self.item_id_embedding.weight
        if tg is None or w.grad is not None or not tg.pending:
            if tg is not None:
                tg.pending = False
            if h_dev is None:
                self.optims.step()
            else:
                self.optims.step_device(h_dev)
            self._norm_tok = None
            return
        if h_dev is None:
            self._rest_optims.step()
        else:
            self._rest_optims.step_device(h_dev)
        tg.adam(self._table_state, norms=self._norm_buf, h_dev=h_dev)
        self._norm_tok = self._norm_token()

    def _norm_token(self):
        from . import engine as _engine
        return (self.item_id_embedding.weight._version, _engine._raw_writes)

    def _norm_valid(self) -> bool:
        return self._norm_tok is not None and self._norm_tok == self._norm_token()

    @torch.no_grad()
    def _refresh_norm(self):
        """_norm_buf[1] = the table's current norm (before a replay whose
        forward reads it, when the table changed outside the fused Adam)."""
        from .rows import slice_norms2
        self._norm_buf.copy_(slice_norms2(self.item_id_embedding.weight.detach(), 0))
        self._norm_tok = self._norm_token()

    def _step_body(self, ids, packing, seg, length, pos, neg, loss_scale=1.0, n_tok=None):
        """Forward, loss and backward of one packed batch; returns the loss.
        ``ids`` = the packed item ids, or (with ``n_tok``) the ids already
        followed by pos and neg (mirec_seq_pack's ids_all)."""
        B = pos.numel()
        if n_tok is None:
            n_tok = ids.numel()
            ids = torch.cat([ids, pos.int(), neg.int()])
        # one lookup for the sequences, positives and negatives (one dense
        # table gradient, no accumulation), one pass of the item tower over
        # positives and negatives together (row-wise: same values).  The
        # table's norm (the loss's only 'emb' parameter term) comes from the
        # same node (one table gradient, written once), and the BPR score /
        # softplus / mean / norm term are one kernel each way.
        x, pn, wnorm = gather_rows_norm(self.item_id_embedding.weight, ids, split=n_tok,
                                        sink=self._tg,
                                        norm=self._norm_buf[1:] if self._norm_valid() else None)
        u = self.forward_user_packed(x, packing, seg, length)
        # the pooled user rows of the last step (B x d; in a captured step
        # the graph's own buffer, rewritten by every replay): parity tests
        self._user_rows = u.detach()
        loss = _BPRRowsLoss.apply(u, self.forward_item(pn), wnorm, self.config["decay"] / B)
        # the backward seed from a kept tensor (no fill kernel per step)
        seed = self.__dict__.get("_loss_seed")
        if seed is None or seed.device != loss.device:
            seed = self._loss_seed = torch.ones((), dtype=loss.dtype, device=loss.device)
        loss.backward(seed if loss_scale == 1.0 else seed * loss_scale)
        return loss

    # ------------------------------------------------------- graph capture
    def packed_ids_static(self, u, capacity: int, pos, neg):
        """packed_ids on the device (mirec_seq_pack, two kernels) for device
        user ids ``u`` [B] into a fixed token capacity (>= the batch's token
        count): rows past the last sequence get item id -1 (a zero row) and
        ``seg`` = B, so every shape is static and the step can be captured.
        The offsets are clamped to the capacity, so a batch that did not fit
        could never make a kernel read past the token buffers (the host sizes
        the capacity from the batch).  Returns (ids_all [capacity + 2B]: the
        token ids then pos and neg as int32, Packing(offsets, padded=True),
        seg [capacity], length [B])."""
        B = u.numel()
        dev = self.device
        items, length_tab = self.seq.items.contiguous(), self.seq.length.contiguous()
        if items.dtype != torch.int32 or length_tab.dtype != torch.int64:
            raise ValueError("SequenceData: int32 items and int64 lengths expected")
        offsets = torch.empty(B + 1, dtype=torch.int32, device=dev)
        length = torch.empty(B, dtype=torch.int64, device=dev)
        ids_all = torch.empty(capacity + 2 * B, dtype=torch.int32, device=dev)
        seg = torch.empty(capacity, dtype=torch.int64, device=dev)
        check(lib.mirec_seq_pack(u.data_ptr(), B, items.data_ptr(), items.shape[1],
                                 length_tab.data_ptr(), pos.data_ptr(), neg.data_ptr(), capacity,
                                 offsets.data_ptr(), length.data_ptr(), ids_all.data_ptr(),
                                 seg.data_ptr(), _lib.stream_handle()), "seq_pack")
        return ids_all, Packing(offsets, None, True), seg, length

    def _graph_step(self, users, pos, neg, hook=None, loss_scale: float = 1.0,
                    table_by_hook: bool | None = None):
        u_host = users.cpu().numpy() if torch.is_tensor(users) else np.asarray(users)
        B = len(u_host)
        n_tok = int(self.seq.length_host[u_host].sum())
        graphs = self.__dict__.setdefault("_graphs", {})
        split = None if hook is None else (loss_scale, table_by_hook)
        fits = [k for k in graphs if k[0] == B and k[2] == self.training and k[1] >= n_tok
                and k[3] == split]
        if fits:
            g = graphs[min(fits, key=lambda k: k[1])]
        else:
            # capacity for this batch and, with margin (mean + 4 sd of a
            # random batch's token count), for the batches after it: one
            # capture serves the run
            lens = self.seq.length_host
            expect = B * float(lens.mean()) + 4.0 * float(lens.std()) * B ** 0.5
            cap = -(-max(n_tok, int(expect)) // 1024) * 1024
            g = graphs[(B, cap, self.training, split)] = _CapturedStep(self, B, cap, u_host,
                                                                       split)
        return g.run(u_host, pos, neg, hook)

    def OneEpoch(self, user, pos, neg):
        B = int(self.config["bpr_batch_size"])
        n = len(user)
        # users on the host: the packed batches are sized without a sync
        user = user.cpu().numpy() if torch.is_tensor(user) else np.asarray(user)
        acc = torch.zeros((), device=self.device)
        for i in range(0, n, B):
            acc += self.stageOne(user[i:i + B], pos[i:i + B], neg[i:i + B])
        return acc / (n // B + 1)

    @torch.no_grad()
    def eval_ratings(self):
        items = self.forward_item(self.item_id_embedding.weight)

        def rate(users):
            x, length = self.sequence_input(users)
            return self.forward_user(x, length) @ items.t()
        return rate

    @torch.no_grad()
    def getUsersRating(self, users):
        return self.eval_ratings()(torch.as_tensor(users, device=self.device))


class _CapturedStep:
    """One SASRec training step (packing, forward, loss, backward, Adam)
    captured in a HIP graph for batch size B and token capacity C, replayed
    every step: the step's ~170 kernel launches cost one graph launch on
    the host.  Everything that changes per step is read from device memory
    when the kernels run: the users / positives / negatives (one staging
    copy), the Adam scalars (mirec_adam_*_dev) and the dropout key base
    (mirec_resnorm_*'s seed_base).  Shapes that depend on the batch are fixed
    by packing into the capacity (packed_ids_static).  Capture runs one eager
    warm-up step on a side stream first (library handles, lazy autograd
    state) and restores the parameters and Adam moments it touched."""

    def __init__(self, model: "SASRec", B: int, capacity: int, u_host, split=None):
        """``split`` = (loss_scale, table_by_hook) captures the data-parallel
        form: graph A (packing, forward, loss x loss_scale, backward) and
        graph B (Adam over the parameters the hook does not step), replayed
        around the hook's collectives."""
        global _SEED_BASE
        self.m, self.B, self.C = model, B, capacity
        self.split = split
        dev = model.device
        # [users | pos | neg | Adam hparams (6 f32 = 3 int64) | seed base];
        # the warm-up runs on the first batch's users (fits the capacity)
        # and first-step Adam scalars
        init = np.zeros(3 * B + 4, dtype=np.int64)
        init[:B] = u_host
        s0 = model.optims.states[0]
        hp0 = _lib.adam_hparams(s0.lr, s0.betas[0], s0.betas[1], s0.eps, 1)
        init[3 * B:3 * B + 3] = np.frombuffer(bytes(hp0), dtype=np.int64)
        self.inbuf = torch.from_numpy(init).to(dev)
        self.stage = [torch.zeros(3 * B + 4, dtype=torch.int64).pin_memory() for _ in range(2)]
        self.events = [None, None]
        self.turn = 0
        if model._tg is not None:
            model._tg.static = True  # the generation is baked into the graph
        pool = model.__dict__.setdefault("_graph_pool", torch.cuda.graph_pool_handle())
        params = list(model.parameters())
        snap = [p.detach().clone() for p in params]
        adam = [(s.exp_avg.clone(), s.exp_avg_sq.clone(), s.n_steps) for s in model.optims]
        for p in params:
            p.grad = None
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        self.graph = torch.cuda.CUDAGraph()
        self.graph_b = torch.cuda.CUDAGraph() if split is not None else None
        try:
            _SEED_BASE = self.inbuf[3 * B + 3:]
            with blas_backend(model.graph_blas()):
                with torch.cuda.stream(side):
                    self._body()  # warm-up (eager, on the side stream)
                    if split is not None:
                        self._body_b()
                torch.cuda.current_stream().wait_stream(side)
                for p in params:
                    p.grad = None
                if split is not None and model._tg is not None:
                    # graph B may not run the fused table Adam that keeps the
                    # norm: the forward reads it from the buffer, refreshed
                    # by run() whenever the table changed
                    model._refresh_norm()
                # the captured forward reads the kept table norm iff it is
                # valid now (the warm-up's fused Adam wrote it)
                self.norm_from_buf = model._norm_valid()
                with torch.cuda.graph(self.graph, pool=pool):
                    self.loss = self._body()
                self.user_rows = model._user_rows  # written by every replay
                # the gradient tensors graph A's backward writes on every
                # replay (AccumulateGrad assigned them during capture; replays
                # never assign .grad again): run() re-attaches them before
                # the hook, which may consume a .grad (the row-sharded Adam
                # sets it to None), so every replay's hook sees them
                self.params = params
                self.grads = [p.grad for p in params]
                if split is not None:
                    tg = model._tg
                    # graph B runs the fused table Adam (which keeps the norm)
                    # iff the table's gradient stays in its sorted form
                    self.fused_b = (not split[1] and tg is not None and tg.pending
                                    and model.item_id_embedding.weight.grad is None)
                    with torch.cuda.graph(self.graph_b, pool=pool):
                        self._body_b()
        finally:
            _SEED_BASE = None
        with torch.no_grad():
            for p, v in zip(params, snap):
                p.copy_(v)
            for s, (a, b, n) in zip(model.optims, adam):
                s.exp_avg.copy_(a)
                s.exp_avg_sq.copy_(b)
                s.n_steps = n

    def _body(self):
        m, B = self.m, self.B
        buf = self.inbuf
        u, pos, neg = buf[:B], buf[B:2 * B], buf[2 * B:3 * B]
        hdev = buf[3 * B:3 * B + 3].view(torch.float32)
        ids_all, packing, seg, length = m.packed_ids_static(u, self.C, pos, neg)
        scale = 1.0 if self.split is None else self.split[0]
        loss = m._step_body(ids_all, packing, seg, length, pos, neg, loss_scale=scale,
                            n_tok=self.C)
        if self.split is None:
            m.optimizer_step(hdev)
        return loss.detach()

    def _group_b(self):
        """The Adam states graph B steps: all but the item table when the
        hook steps it (routed exchange / row-sharded Adam), else all."""
        return self.m._rest_optims if self.split[1] else self.m.optims

    def _body_b(self):
        B = self.B
        hdev = self.inbuf[3 * B:3 * B + 3].view(torch.float32)
        if self.split[1]:
            self.m._rest_optims.step_device(hdev)
        else:  # the table too: fused from its sorted gradient, or densely
            self.m.optimizer_step(hdev)

    def run(self, u_host, pos, neg, hook=None):
        B = self.B
        k = self.turn
        self.turn ^= 1
        if self.events[k] is not None:
            self.events[k].synchronize()  # staging buffer k's last copy is done
        st = self.stage[k].numpy()
        st[:B] = u_host
        on_dev = [torch.is_tensor(t) and t.is_cuda for t in (pos, neg)]
        for j, (t, dv) in enumerate(((pos, on_dev[0]), (neg, on_dev[1]))):
            if not dv:
                st[(j + 1) * B:(j + 2) * B] = np.asarray(t.cpu() if torch.is_tensor(t) else t)
        if self.split is None or not self.split[1]:
            hp = self.m.optims.next_shared_hparams(require_grad=False)
        else:
            hp = self.m._rest_optims.next_shared_hparams(require_grad=False)
        st[3 * B:3 * B + 3] = np.frombuffer(bytes(hp), dtype=np.int64)
        st[3 * B + 3] = int(torch.randint(0, 2 ** 62, (1,)).item())  # torch's CPU generator
        self.inbuf.copy_(self.stage[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        pair = (on_dev[0] and on_dev[1] and pos.dtype == torch.int64 and neg.dtype == torch.int64
                and pos.dim() == 1 and neg.dim() == 1 and pos._base is not None
                and pos._base is neg._base and pos._base.is_contiguous()
                and neg.data_ptr() == pos.data_ptr() + 8 * B)
        if pair:  # one [pos ; neg] block (sample_pairs): one copy
            self.inbuf[B:3 * B].copy_(pos._base.view(-1)[:2 * B])
        else:
            for j, (t, dv) in enumerate(((pos, on_dev[0]), (neg, on_dev[1]))):
                if dv:  # device ids: copied after the staging copy (stream order)
                    self.inbuf[(j + 1) * B:(j + 2) * B].copy_(t)
        m = self.m
        if self.norm_from_buf and not m._norm_valid():
            m._refresh_norm()  # the table changed outside the step
        _note_raw_write()
        self.graph.replay()
        if self.split is not None:
            if m._tg is not None:
                m._tg.pending = True  # the replayed backward left S / coef
            for p, g in zip(self.params, self.grads):
                p.grad = g
            hook()
            if m._tg is not None:
                m._tg.pending = False
            self.graph_b.replay()
            _note_raw_write()
            # the fused table Adam of graph B wrote the next norm; otherwise
            # the next run refreshes it
            m._norm_tok = m._norm_token() if self.fused_b else None
            return self.loss.clone()
        if m._tg is not None:  # the replayed fused Adam wrote the next norm
            m._norm_tok = m._norm_token()
        return self.loss.clone()
