"""SASRec (model/sasrec.py:54-502) — the self-attention block on MFMA.

In scope: the per-layer block of sasrec.py:385-397
(pre-LN → causal multi-head self-attention → dropout → residual + ReLU →
LN → Linear → dropout → residual), the masked mean pool over the first
`length` positions (:399-413), the item MLP tower (:415-421), the BPR loss
with the reference's embedding-norm term (:423-435) and OneEpoch (:437-474).
The attention core softmax(QKᵀ/√d_h + causal)·V and its backward are one
HIP launch each (csrc/attention.hip, f32 MFMA); the projections, LayerNorm
and FFN are library GEMMs, and the dropout / residual / ReLU /
LayerNorm tail of each stage is one fused row kernel (csrc/resnorm.hip).
Out of scope: the proprietary text / feature towers of the initial item
embedding (:82-209): items start from an id embedding (N(0, 1), :205).
The reference hard-codes 8 heads (:211); `heads` is a parameter here
(BASELINE config C4 uses 2).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import check, lib
from .engine import AdamGroup, AdamState
from .linear import Linear, blas_backend, linear
from .rows import gather_rows


# Optional per-launch timing (tools/bench_sasrec.py): a list receiving
# (kind, start_event, end_event, (B, T, heads, head_dim), offsets or None);
# packed launches have T = -1 and their int32 offsets.
ATTN_EVENTS = None


def _timed(kind, shape, launch, offsets=None):
    ev = ATTN_EVENTS
    if ev is None:
        return launch()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    r = launch()
    e.record()
    ev.append((kind, s, e, shape, offsets))
    return r


class _CausalAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads: int):
        B, T, d3 = qkv.shape
        d = d3 // 3
        qkv = qkv.contiguous()
        out = torch.empty(B, T, d, dtype=qkv.dtype, device=qkv.device)
        _timed("fwd", (B, T, heads, d // heads), lambda: check(lib.mirec_attention_fwd(
            qkv.data_ptr(), B, T, heads, d // heads, out.data_ptr(), _lib.stream_handle()),
            "attention_fwd"))
        ctx.save_for_backward(qkv)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        (qkv,) = ctx.saved_tensors
        B, T, d3 = qkv.shape
        dh = d3 // 3 // ctx.heads
        dqkv = torch.empty_like(qkv)
        dout = dout.contiguous()
        _timed("bwd", (B, T, ctx.heads, dh), lambda: check(lib.mirec_attention_bwd(
            qkv.data_ptr(), dout.data_ptr(), B, T, ctx.heads, dh, dqkv.data_ptr(),
            _lib.stream_handle()), "attention_bwd"))
        return dqkv, None


class _CausalAttentionVarlen(torch.autograd.Function):
    """Packed sequences: qkv [n_tok, 3d], sequence b = rows offsets[b] ..
    offsets[b+1]-1 (mirec_attention_varlen_*)."""

    @staticmethod
    def forward(ctx, qkv, offsets, heads: int):
        n, d3 = qkv.shape
        d = d3 // 3
        B = offsets.numel() - 1
        qkv = qkv.contiguous()
        out = torch.empty(n, d, dtype=qkv.dtype, device=qkv.device)
        _timed("fwd", (B, -1, heads, d // heads), lambda: check(lib.mirec_attention_varlen_fwd(
            qkv.data_ptr(), offsets.data_ptr(), B, heads, d // heads, out.data_ptr(),
            _lib.stream_handle()), "attention_varlen_fwd"), offsets)
        ctx.save_for_backward(qkv, offsets)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, offsets = ctx.saved_tensors
        n, d3 = qkv.shape
        B = offsets.numel() - 1
        dh = d3 // 3 // ctx.heads
        dqkv = torch.empty_like(qkv)
        dout = dout.contiguous()
        _timed("bwd", (B, -1, ctx.heads, dh), lambda: check(lib.mirec_attention_varlen_bwd(
            qkv.data_ptr(), dout.data_ptr(), offsets.data_ptr(), B, ctx.heads, dh,
            dqkv.data_ptr(), _lib.stream_handle()), "attention_varlen_bwd"), offsets)
        return dqkv, None, None


def _ptr(t):
    return 0 if t is None else t.data_ptr()


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
    def forward(ctx, res, z, bias, gamma, beta, relu: bool, p: float, eps: float, norm: bool):
        n, d = z.shape
        pure = res is None and bias is None and not relu and p == 0
        seed = _dropout_seed(p)
        out = None if pure else torch.empty_like(z)
        y = mean = rstd = None
        if norm:
            y = torch.empty_like(z)
            mean = torch.empty(n, dtype=z.dtype, device=z.device)
            rstd = torch.empty_like(mean)
        check(lib.mirec_resnorm_fwd(_ptr(res), z.data_ptr(), _ptr(bias), _ptr(gamma),
                                    _ptr(beta), n, d, int(relu), float(p), seed, float(eps),
                                    _ptr(out), _ptr(y), _ptr(mean), _ptr(rstd),
                                    _lib.stream_handle()), "resnorm_fwd")
        ctx.save_for_backward(z if pure else out, mean, rstd, gamma)
        ctx.cfg = (relu, float(p), seed, res is not None, bias is not None, norm)
        ctx.set_materialize_grads(False)
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
                                    _ptr(d_res), _ptr(d_z), _ptr(work), _ptr(d_gamma),
                                    _ptr(d_beta), _ptr(d_bias), _lib.stream_handle()),
              "resnorm_bwd")
        if norm and g_y is None:  # y unused downstream: no LayerNorm gradients
            d_gamma = torch.zeros_like(gamma) if need[3] and gamma is not None else None
            d_beta = torch.zeros(d, dtype=out.dtype, device=out.device) if need[4] else None
        return d_res, d_z, d_bias, d_gamma, d_beta, None, None, None, None


def resnorm(res, z, bias=None, norm: nn.LayerNorm | None = None, relu: bool = False,
            p: float = 0.0):
    """(out, y) of _ResNorm for rows of width d = z.shape[-1] (any leading
    shape); ``norm`` an nn.LayerNorm over d or None."""
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
    out, y = _ResNorm.apply(r2, z2, bias, gamma, beta, relu, p, eps, norm is not None)
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
        [B+1] (sequence b = rows offsets[b] .. offsets[b+1]-1)."""
        return self.out_proj(self.core(x, offsets))

    def core(self, x, offsets=None):
        """The heads' outputs before the out-projection."""
        qkv = linear(x, self.in_proj_weight, self.in_proj_bias)
        if offsets is None:
            return _CausalAttention.apply(qkv, self.heads)
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
        _, y = resnorm(None, x, norm=self.attn_norm_layers[0])
        res = x
        L = self.num_layers
        for i in range(L):
            attn = self.attn_layers[i]
            z = linear(attn.core(y, offsets), attn.out_proj.weight)
            h, y = resnorm(res, z, attn.out_proj.bias, self.ffn_norm_layers[i], relu=True, p=p)
            ffn = self.ffn_layers[i]
            f = linear(y, ffn.weight)
            nxt = self.attn_norm_layers[i + 1] if i + 1 < L else None
            res, y = resnorm(h, f, ffn.bias, nxt, p=p)
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
        the sequence of every row.  Padding positions never reach a real
        position under the causal mask and are excluded from the pool, so
        this equals forward_user on the padded batch while skipping them."""
        x = self.blocks(x, offsets)
        pooled = torch.zeros(length.numel(), x.shape[1], dtype=x.dtype, device=x.device)
        pooled = pooled.index_add(0, seg, x)
        return pooled / length.to(x.dtype).unsqueeze(1)

    def packed_input(self, users):
        """(x [n_tok, d], offsets [B+1] int32, seg [n_tok], length [B]) of the
        users' sequences.  The token count is taken from the host copy of
        the lengths (host ``users``: no device synchronisation)."""
        ids, offsets, seg, length = self.packed_ids(users)
        return gather_rows(self.item_id_embedding.weight, ids), offsets, seg, length

    def packed_ids(self, users):
        """packed_input's item ids [n_tok] (int32) instead of their rows."""
        if torch.is_tensor(users) and users.is_cuda:
            u_host = users.cpu().numpy()
        else:
            u_host = np.asarray(users)
        lens_h = self.seq.length_host[u_host]
        n_tok = int(lens_h.sum())
        dev = self.device
        u = self._upload(u_host)
        length = self.seq.length[u]
        offsets = torch.zeros(len(u_host) + 1, dtype=torch.int32, device=dev)
        offsets[1:] = torch.cumsum(length, 0).to(torch.int32)
        seg = torch.repeat_interleave(torch.arange(len(u_host), device=dev), length,
                                      output_size=n_tok)
        pos = torch.arange(n_tok, device=dev) - offsets[seg].long()
        return self.seq.items[u[seg], pos], offsets, seg, length

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

    def forward_item(self, x):
        """sasrec.py:415-421."""
        for lin in self.item_linears:
            x = lin(x).relu()
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

    def stageOne(self, users, pos, neg, grad_hook=None, loss_scale: float = 1.0):
        """One BPR step on packed sequences.  ``loss_scale`` scales the
        gradient (1/world_size under data parallelism); ``grad_hook`` runs
        between backward and Adam (DenseGradDataParallel's all-reduce).
        The projections run on the BLAS backend of config "blas" (default
        rocBLAS: the step is host-bound and rocBLAS launches cheaper)."""
        with blas_backend(self.config.get("blas", "cublas")):
            return self._stage_one(users, pos, neg, grad_hook, loss_scale)

    def _stage_one(self, users, pos, neg, grad_hook, loss_scale):
        for p in self.parameters():
            p.grad = None
        pos, neg = (torch.as_tensor(t).to(self.device) for t in (pos, neg))
        ids, offsets, seg, length = self.packed_ids(users)
        n_tok, B = ids.numel(), pos.numel()
        # one lookup for the sequences, positives and negatives (one dense
        # table gradient, no accumulation), one pass of the item tower over
        # positives and negatives together (row-wise: same values)
        rows = gather_rows(self.item_id_embedding.weight, torch.cat([ids, pos.int(), neg.int()]))
        x, pn = rows.split([n_tok, 2 * B])
        u = self.forward_user_packed(x, offsets, seg, length)
        pe, ne = self.forward_item(pn).split(B)
        loss = self.loss(u, pe, ne)
        (loss * loss_scale if loss_scale != 1.0 else loss).backward()
        if grad_hook is not None:
            grad_hook()
        self.optims.step()
        return loss.detach()

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
