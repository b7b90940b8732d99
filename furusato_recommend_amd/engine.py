"""LightGCN propagation + BPR training engine (device side orchestration).

One training step (the reference's ``stageOne``, model/lgcn.py:127-133, on
top of ``bpr_loss`` :98-118 and ``forward`` :78-86) runs as ~2L+8 HIP
launches with no host synchronisation:

  frontier (3-4)          S = batch nodes, F1 = S ∪ N(S) as byte maps and
                          row lists
  forward  (L [+1])       x~_0 = dinv ⊙ E (skipped when the previous step's
                          fused update already wrote it), x_l = Â x_{l-1};
                          acc = x_0 + ... + x_L; out = acc/(L+1).  Every
                          layer gathers pre-scaled rows x~ = dinv ⊙ x written
                          by the previous epilogue; layer L runs on S only,
                          layer L-1 on F1 only (pruning).
  BPR      (3 + sort)     scores, softplus, loss; sorted (node, occurrence)
                          pairs → per-node gradient seeds d = dL/d out /(L+1)
                          and the reg-gradient seed.
  backward (L launches)   Horner: g_L = d, g_l = d + Â g_{l+1} (Â symmetric:
                          the backward SpMM is the forward kernel on the
                          same CSR).  The first backward layer gathers only
                          the seeded neighbours (IN_SPARSE: slot[j] >= 0) and
                          is written on F1 only; the second skips neighbours
                          outside F1; the last one adds the reg seed and
                          applies Adam to E in its epilogue, so the dense
                          gradient is never written to HBM; it also writes
                          dinv ⊙ E_new, the next step's x~_0.
  reset    (1)            slot[] back to -1 for the touched nodes.

For data parallelism (dist.py) the ranks exchange their gradient seeds
before the backward (sparse mode), or the last layer writes the dense
gradient and the caller all-reduces it before ``adam_step`` (dense mode).
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from ._lib import (IN_NONE, IN_PRESCALED, IN_RAW, IN_SPARSE, Prop, adam_hparams,
                   check, lib, ptr)
from .graph import Graph


def prop_launch_bytes(in_mode: int, n_nodes: int, nnz: int, dim: int, *, slot=False,
                      xs_out=False, addend=False, out=False, adam=False) -> int:
    """Algorithmic HBM bytes of one mirec_propagate launch:
    every operand the launch must read or write, each exactly once."""
    N, D = n_nodes, dim
    row = N * D * 4
    b = (N + 1) * 8 + N * 4                       # rowptr (int64), dinv_i
    if in_mode == IN_PRESCALED:
        b += nnz * (D * 4 + 4)                    # neighbour rows + col
    elif in_mode == IN_RAW:
        b += nnz * (D * 4 + 4 + 4)                # + dinv_j per entry
    elif in_mode == IN_SPARSE:
        b += nnz * (4 + 4 + 4)                    # col, dinv_j, slot_j
    if slot:
        b += N * 4                                # slot_i
    b += row * (int(xs_out) + int(addend) + int(out))
    if adam:
        b += 6 * row                              # param/m/v read + write
    return b


# Generation counter of raw-pointer writes to parameter tables (kernels do
# not bump torch's version counter); part of the engine's prescale token.
_raw_writes = 0


def _note_raw_write():
    global _raw_writes
    _raw_writes += 1


class AdamState:
    """torch.optim.Adam state for one dense parameter, in torch's layout."""

    def __init__(self, param: torch.Tensor, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        self.param = param
        self.lr = float(lr)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.n_steps = 0
        self.exp_avg = torch.zeros_like(param)
        self.exp_avg_sq = torch.zeros_like(param)
        # set by a data-parallel wrapper that updates this state on its own
        # row shard only (the other rows' moments are stale until gathered)
        self.stale_rows = False

    def next_hparams(self):
        self.n_steps += 1
        return adam_hparams(self.lr, self.betas[0], self.betas[1], self.eps, self.n_steps)

    # torch.optim-style surface for the differentiable path (reference
    # stageOne: optim.zero_grad(); loss.backward(); optim.step()).
    def zero_grad(self, set_to_none: bool = True):
        if self.param.grad is not None:
            if set_to_none:
                self.param.grad = None
            else:
                self.param.grad.zero_()

    @torch.no_grad()
    def step(self):
        g = self.param.grad
        if g is None:
            return
        hp = self.next_hparams()
        _note_raw_write()
        check(lib.mirec_adam_dense(self.param.data_ptr(), g.contiguous().data_ptr(),
                                   self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                   self.param.numel(), ctypes.byref(hp), _lib.stream_handle()),
              "adam_dense")

    def _launch(self, hp):
        g = self.param.grad.contiguous()
        check(lib.mirec_adam_dense(self.param.data_ptr(), g.data_ptr(),
                                   self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                   self.param.numel(), ctypes.byref(hp), _lib.stream_handle()),
              "adam_dense")

    def state_dict(self, param_id: int = 0) -> dict:
        """Same structure as torch.optim.Adam.state_dict() for one param."""
        if self.stale_rows:
            raise RuntimeError("Adam moments are sharded over the data-parallel ranks: call "
                               "gather_optimizer_state() on every rank before state_dict()")
        return {
            "state": {param_id: {"step": torch.tensor(float(self.n_steps)),
                                 "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}},
            "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                              "weight_decay": 0, "amsgrad": False, "maximize": False,
                              "foreach": None, "capturable": False, "differentiable": False,
                              "fused": None, "params": [param_id]}],
        }

    def load_state_dict(self, sd: dict) -> None:
        st = next(iter(sd["state"].values())) if sd["state"] else None
        if st is not None:
            self.n_steps = int(float(st["step"]))
            self.exp_avg.copy_(st["exp_avg"])
            self.exp_avg_sq.copy_(st["exp_avg_sq"])
        g = sd["param_groups"][0]
        self.lr, self.betas, self.eps = float(g["lr"]), tuple(g["betas"]), float(g["eps"])


class AdamGroup:
    """Steps a model's AdamStates together: tensors of at least LARGE
    elements with the float4 dense kernel, all the others in one
    mirec_adam_multi launch per distinct (step, lr, betas, eps) — instead of
    one launch (and one host round of Python) per parameter."""

    LARGE = 1 << 20

    def __init__(self, states):
        self.states = list(states)

    def __iter__(self):
        return iter(self.states)

    def __len__(self):
        return len(self.states)

    def zero_grad(self, set_to_none: bool = True):
        for s in self.states:
            s.zero_grad(set_to_none)

    @torch.no_grad()
    def step(self):
        groups = {}
        for s in self.states:
            if s.param.grad is None:
                continue
            hp = s.next_hparams()
            if s.param.numel() >= self.LARGE:
                s._launch(hp)
                continue
            key = (s.n_steps, s.lr, s.betas, s.eps)
            groups.setdefault(key, (hp, []))[1].append(s)
        if not groups and not any(s.param.grad is not None for s in self.states):
            return
        _note_raw_write()
        for hp, members in groups.values():
            n = len(members)
            grads = [m.param.grad.contiguous() for m in members]
            arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
            numel = (ctypes.c_int64 * n)(*[m.param.numel() for m in members])
            check(lib.mirec_adam_multi(n, arr([m.param for m in members]), arr(grads),
                                       arr([m.exp_avg for m in members]),
                                       arr([m.exp_avg_sq for m in members]), numel,
                                       ctypes.byref(hp), _lib.stream_handle()), "adam_multi")

    # -- graph-captured steps: the scalars live in device memory ------------
    def next_shared_hparams(self, require_grad: bool = True):
        """Advance every state (all must share lr / betas / eps / step count
        and, with require_grad, have a gradient) and return the one hparams
        struct of this step — what a captured step reads through
        step_device."""
        keys = {(s.n_steps, s.lr, s.betas, s.eps) for s in self.states}
        if len(keys) != 1 or (require_grad and any(s.param.grad is None for s in self.states)):
            raise RuntimeError("device-scalar Adam needs one shared step for every parameter")
        hps = [s.next_hparams() for s in self.states]
        return hps[0]

    @torch.no_grad()
    def step_device(self, h_dev: torch.Tensor):
        """The update of step() with the hyper-parameters read from ``h_dev``
        (a device buffer of one mirec_adam_hparams_t) when the kernels run:
        capturable in a HIP graph.  Does not advance the host step counts
        (next_shared_hparams does, once per replay)."""
        _note_raw_write()
        large = [s for s in self.states if s.param.numel() >= self.LARGE]
        small = [s for s in self.states if s.param.numel() < self.LARGE]
        for s in large:
            g = s.param.grad.contiguous()
            check(lib.mirec_adam_dense_dev(s.param.data_ptr(), g.data_ptr(), s.exp_avg.data_ptr(),
                                           s.exp_avg_sq.data_ptr(), s.param.numel(),
                                           h_dev.data_ptr(), _lib.stream_handle()),
                  "adam_dense_dev")
        if small:
            n = len(small)
            grads = [m.param.grad.contiguous() for m in small]
            arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
            numel = (ctypes.c_int64 * n)(*[m.param.numel() for m in small])
            check(lib.mirec_adam_multi_dev(n, arr([m.param for m in small]), arr(grads),
                                           arr([m.exp_avg for m in small]),
                                           arr([m.exp_avg_sq for m in small]), numel,
                                           h_dev.data_ptr(), _lib.stream_handle()),
                  "adam_multi_dev")


class PropagationEngine:
    """Owns the per-model scratch buffers and issues the HIP launches.

    ``prune`` (default on) enables frontier pruning: with S the batch's
    nodes and F1 = S ∪ N(S) (mirec_frontier), forward layer L is computed on
    S only and layer L-1 on F1 only (the loss reads the layer mean only on
    S), and the first two backward layers skip the rows / neighbours that
    are exactly zero.  Loss, gradient and update are the dense pass's up to
    fp32 summation order; ``prune=False`` runs every layer on every row."""

    def __init__(self, graph: Graph, dim: int, n_layers: int, max_batch: int,
                 prune: bool = True):
        if dim not in _lib.SUPPORTED_DIMS:
            raise ValueError(f"recdim={dim} not supported by the HIP engine "
                             f"(supported: {_lib.SUPPORTED_DIMS})")
        if graph.device.type != "cuda":
            raise RuntimeError("PropagationEngine needs a HIP device (no CPU fallback)")
        self.g = graph
        self.dim = int(dim)
        self.L = int(n_layers)
        self.max_batch = int(max_batch)
        self.prune = bool(prune)
        dev = graph.device
        N, D = graph.n_nodes, self.dim
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.acc = torch.empty(N, D, **f32)       # layer sum, then out = acc/(L+1)
        self.x0s = torch.empty(N, D, **f32) if self.L > 0 else None  # dinv ⊙ E
        self.xs = [torch.empty(N, D, **f32), torch.empty(N, D, **f32)] if self.L > 1 else \
            [torch.empty(N, D, **f32)] if self.L == 1 else []
        self.slot = torch.full((N,), -1, **i32)
        words = (N + 15) // 16 * 4  # 16-byte rows (mask_compact reads 16 B per thread)
        # S and S ∪ N(S) byte maps (int32-backed), adjacent: cleared together
        self._bm = torch.zeros(2, words, **i32)
        self.bm_self, self.bm_hop = self._bm[0], self._bm[1]
        self.self_list = torch.zeros(3 * self.max_batch, **i32)  # S, deduplicated
        self.self_count = torch.zeros(1, **i32)
        self._self_cap = 0
        # S and F1 as row lists split by degree (narrow: <= narrow_max,
        # gathered G rows per wave; wide: one workgroup per row)
        cap = N if self.prune else 1
        self.s_lists = (torch.zeros(cap, **i32), torch.zeros(cap, **i32))
        self.hop_lists = (torch.zeros(cap, **i32), torch.zeros(cap, **i32))
        self.list_counts = torch.zeros(4, **i32)  # S narrow, S wide, F1 narrow, F1 wide
        # tuning switches (tools/bench_variants.py)
        self.use_hop_list = True      # F1 launches walk hop_list (else: byte map)
        self.reuse_prescaled = True   # fused update writes the next x~_0
        # first backward layer's neighbour filter: "slot" (one dependent load;
        # best for one batch), "bytemap" (S byte map, then the slot of the
        # hits), "dense" (seed rows scattered into a zero [N, D] table and
        # gathered as a byte-map-filtered PRESCALED input) or "auto"
        self.sparse_filter = "auto"
        self._masks_ready = False
        # rows of degree <= narrow_max are gathered one per lane group
        self.narrow_max = 64
        B3 = 3 * self.max_batch
        self.seed_p = torch.empty(B3, D, **f32)
        self.seed_e = torch.empty(B3, D, **f32)
        self.coef = torch.empty(self.max_batch, **f32)
        self.softplus = torch.empty(self.max_batch, **f32)
        self.reg = torch.empty(self.max_batch, **f32)
        self.keys = torch.empty(B3, **i32)
        self.vals = torch.empty(B3, **i32)
        self.keys_sorted = torch.empty(B3, **i32)
        self.loss = torch.zeros(1, **f32)
        self.partial = graph.partial_buffer(D)
        self._ws = None
        self._ws_bytes = 0
        self._ensure_ws(self.max_batch)
        # Optional per-launch timing of the propagation kernel (bench.py):
        # list of (start, end, (in_mode, in_masked, row_masked), bytes).
        self.prop_events = None
        self._seeds = None
        self._merged = None
        # (data_ptr, _version) of the table x0s = dinv ⊙ E was last written
        # for by a fused-Adam backward (which emits it for free); forward()
        # skips the prescale pass when the table is unchanged since.
        self._x0s_token = None
        # token of the table whose FULL layer mean ``acc`` holds (None after a
        # pruned forward or any update): repeated getUsersRating calls of one
        # evaluation reuse it instead of re-propagating
        self._acc_full = None

    # ------------------------------------------------------------ internals
    def _ensure_ws(self, batch: int):
        nb = ctypes.c_size_t(0)
        check(lib.mirec_bpr_seed_workspace(batch, self.g.n_nodes, ctypes.byref(nb)),
              "bpr_seed_workspace")
        if nb.value > self._ws_bytes:
            self._ws = torch.empty(nb.value, dtype=torch.uint8, device=self.g.device)
            self._ws_bytes = nb.value

    def _prop(self, *, in_mode, x_in=None, seed_in=None, seed=None, addend=None, seed2=None,
              divisor=1.0, out=None, xs_out=None, adam=None, param=None, graph=None,
              row_mask=None, in_mask=None, row_list=None, row_count=None, row_list_cap=0,
              out_mask=None, wide_list=None, wide_count=None):
        g = graph or self.g
        p = Prop()
        p.dim = self.dim
        p.in_mode = in_mode
        p.x_in = ptr(x_in)
        p.slot = self.slot.data_ptr() if (seed_in is not None or seed is not None
                                          or seed2 is not None) else None
        p.seed_in = ptr(seed_in)
        p.seed = ptr(seed)
        p.addend = ptr(addend)
        p.seed2 = ptr(seed2)
        p.divisor = float(divisor)
        p.out = ptr(out)
        p.xs_out = ptr(xs_out)
        if adam is not None:
            state, hp = adam
            p.param = param.data_ptr()
            p.exp_avg = state.exp_avg.data_ptr()
            p.exp_avg_sq = state.exp_avg_sq.data_ptr()
            p.adam = hp
        part = g.partial_buffer(self.dim)
        p.partial = ptr(part)
        p.row_mask = ptr(row_mask)
        p.in_mask = ptr(in_mask)
        p.out_mask = ptr(out_mask)
        p.row_list = ptr(row_list)
        p.row_count = ptr(row_count)
        p.row_list_cap = int(row_list_cap)
        p.wide_list = ptr(wide_list)
        p.wide_count = ptr(wide_count)
        p.narrow_max = int(self.narrow_max)
        ev = self.prop_events
        if ev is not None:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        check(lib.mirec_propagate(g.csr_ptr(), ctypes.byref(p), _lib.stream_handle()),
              "propagate")
        if ev is not None:
            e.record()
            kind = (in_mode, in_mask is not None, row_mask is not None, out_mask is not None)
            ev.append((s, e, kind, self.launch_bytes(p, g)))

    def launch_bytes(self, p: Prop, g: Graph) -> int:
        """Algorithmic bytes of a launch over every row.  With an out_mask the
        `out`/addend streams are excluded (the caller adds 2·|mask|·D·4 from
        the measured mask size)."""
        om = bool(p.out_mask)
        return prop_launch_bytes(p.in_mode, g.n_nodes, g.nnz, self.dim,
                                 slot=bool(p.slot and (p.seed or p.seed2)),
                                 xs_out=bool(p.xs_out), addend=bool(p.addend) and not om,
                                 out=bool(p.out) and not om, adam=bool(p.param))

    def compute_frontier(self, users=None, pos=None, neg=None, keys=None, n_keys: int = 0):
        """bm_self = S, bm_hop = S ∪ N(S) for a triple batch or a key list;
        self_list = S deduplicated, hop_list = F1 as a row list (pruning)."""
        g = self.g
        # the row-list counters of the mask_compact calls below are cleared by
        # the frontier's clear launch (one launch for maps, S count, counters)
        lists = self.prune and self.use_hop_list
        zc, nz = (self.list_counts.data_ptr(), 4) if lists else (None, 0)
        if keys is not None:
            n = int(n_keys)
            if self.self_list.shape[0] < n:
                self.self_list = torch.zeros(n, dtype=torch.int32, device=g.device)
            check(lib.mirec_frontier(g.csr_ptr(), keys.data_ptr(), n, None, None, None,
                                     0, g.n_users, self.bm_self.data_ptr(),
                                     self.bm_hop.data_ptr(), self.self_list.data_ptr(),
                                     self.self_count.data_ptr(), zc, nz, _lib.stream_handle()),
                  "frontier")
            self._self_cap = n
        else:
            B = int(users.shape[0])
            if B > self.max_batch:
                raise ValueError(f"batch {B} > engine max_batch {self.max_batch}")
            check(lib.mirec_frontier(g.csr_ptr(), None, 0, users.data_ptr(), pos.data_ptr(),
                                     neg.data_ptr(), B, g.n_users,
                                     self.bm_self.data_ptr(), self.bm_hop.data_ptr(),
                                     self.self_list.data_ptr(), self.self_count.data_ptr(),
                                     zc, nz, _lib.stream_handle()), "frontier")
            self._self_cap = 3 * B
        if lists:
            # S and F1 compacted in one launch, the degree split from a static
            # bitmap (mirec_mask_compact_pair; counters zeroed by the frontier)
            check(lib.mirec_mask_compact_pair(self.bm_self.data_ptr(), self.bm_hop.data_ptr(),
                                              self._wide_bits().data_ptr(), g.n_nodes,
                                              self.s_lists[0].data_ptr(),
                                              self.s_lists[1].data_ptr(),
                                              self.hop_lists[0].data_ptr(),
                                              self.hop_lists[1].data_ptr(),
                                              self.list_counts.data_ptr(), _lib.stream_handle()),
                  "mask_compact_pair")
        self._masks_ready = True

    def _wide_bits(self) -> torch.Tensor:
        """Bit v of word v // 32: node v's degree > narrow_max (the row lists'
        narrow / wide split), built once per graph and narrow_max."""
        key = int(self.narrow_max)
        wb = getattr(self, "_wide_bits_cache", None)
        if wb is not None and wb[0] == key:
            return wb[1]
        g = self.g
        rp = g.rowptr
        n = g.n_nodes
        wide = (rp[1:n + 1] - rp[:n]) > key
        words = (n + 31) // 32
        bits = torch.zeros(words * 32, dtype=torch.int64, device=wide.device)
        bits[:n] = wide.to(torch.int64)
        shifts = torch.arange(32, dtype=torch.int64, device=wide.device)
        w = (bits.view(words, 32) << shifts).sum(1)        # < 2^32
        w = torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)
        self._wide_bits_cache = (key, w.contiguous())
        return self._wide_bits_cache[1]

    def _lists(self, k, bm, lists, cap):
        if not self.use_hop_list:
            return dict(row_mask=bm)
        c = self.list_counts
        return dict(row_mask=bm, row_list=lists[0], row_count=c[2 * k], row_list_cap=cap,
                    wide_list=lists[1], wide_count=c[2 * k + 1])

    def _dense_seeds(self, seed_p, clear: int):
        """Write (clear=0) or zero (clear=1) the pre-scaled seed rows of S in an
        all-zero [N, D] table (sparse_filter == "dense")."""
        if getattr(self, "seed_dense", None) is None:
            self.seed_dense = torch.zeros(self.g.n_nodes, self.dim, dtype=torch.float32,
                                          device=self.g.device)
        check(lib.mirec_seed_dense(self.self_list.data_ptr(), self.self_count.data_ptr(),
                                   self._self_cap, self.slot.data_ptr(), self.g.dinv.data_ptr(),
                                   seed_p.data_ptr(), self.dim, self.seed_dense.data_ptr(),
                                   int(clear), _lib.stream_handle()), "seed_dense")
        return self.seed_dense

    def _sparse_filter(self):
        f = self.sparse_filter
        if f == "auto":
            f = "bytemap" if self._self_cap > 3 * self.max_batch else "slot"
        return self.bm_self if f == "bytemap" else None

    def static_row_lists(self, bm: torch.Tensor) -> dict:
        """Launch arguments restricting a propagation to the rows whose byte in
        ``bm`` (uint8-viewable, [>= n_rows]) is set: the byte map plus its
        narrow / wide row lists, built once (a fixed row set, e.g. a
        data-parallel rank's shard)."""
        g = self.g
        N = g.n_nodes
        dev = g.device
        nl = torch.zeros(max(N, 1), dtype=torch.int32, device=dev)
        wl = torch.zeros(max(N, 1), dtype=torch.int32, device=dev)
        cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        check(lib.mirec_mask_compact(g.csr_ptr(), bm.data_ptr(), int(self.narrow_max),
                                     nl.data_ptr(), cnt[0].data_ptr(), wl.data_ptr(),
                                     cnt[1].data_ptr(), 0, _lib.stream_handle()), "mask_compact")
        return dict(row_mask=bm, row_list=nl, row_count=cnt[0], row_list_cap=N,
                    wide_list=wl, wide_count=cnt[1])

    def _self_rows(self):
        return self._lists(0, self.bm_self, self.s_lists, min(self._self_cap, self.g.n_nodes))

    def _hop_rows(self):
        return self._lists(1, self.bm_hop, self.hop_lists, self.g.n_nodes)

    @staticmethod
    def _token(emb: torch.Tensor):
        return (emb.data_ptr(), emb._version, _raw_writes)

    def invalidate_prescaled(self):
        """Forget the cached dinv ⊙ E.  Needed only after writing the table
        through ``.data`` (invisible to the tensor's version counter) between
        training steps; in-place torch ops, ``load_state_dict`` and
        re-assignment are detected.  Also drops the cached full propagation
        (forward_cached)."""
        self._x0s_token = None
        self._acc_full = None

    def mark_prescaled(self, emb: torch.Tensor):
        """x0s holds dinv ⊙ emb on every row (written piecewise by the
        caller, e.g. the sharded data-parallel unpack): the next forward
        skips its prescale pass."""
        self._x0s_token = self._token(emb)
        self._acc_full = None

    def prescale(self, x: torch.Tensor, out: torch.Tensor):
        check(lib.mirec_prescale(x.data_ptr(), self.g.dinv.data_ptr(), self.g.n_nodes, self.dim,
                                 out.data_ptr(), _lib.stream_handle()), "prescale")

    # ------------------------------------------------------------- forward
    def forward(self, emb: torch.Tensor, pruned: bool = False) -> torch.Tensor:
        """out = (x_0 + ... + x_L)/(L+1), x_l = Â x_{l-1} (model/lgcn.py:78-86).

        ``pruned`` (after compute_frontier): rows outside the frontier are not
        computed (valid only on S).  Returns the engine's ``acc`` buffer
        (valid until the next call)."""
        L = self.L
        self._acc_full = None
        if L == 0:
            self.acc.copy_(emb)
            self._acc_full = self._token(emb)
            return self.acc
        if pruned and not self._masks_ready:
            raise RuntimeError("forward(pruned=True) needs compute_frontier() first")
        if self._x0s_token != self._token(emb):
            self.prescale(emb, self.x0s)
            self._x0s_token = self._token(emb)
        for l in range(1, L + 1):
            last = l == L
            rows = {}
            if pruned and l == L:      # S: the deduplicated batch-node list
                rows = self._self_rows()
            elif pruned and l == L - 1:  # F1 = S ∪ N(S)
                rows = self._hop_rows()
            if pruned and l == L - 2:
                # the layer sum is read next by layer L-1, on F1 rows only
                rows["out_mask"] = self.bm_hop
            self._prop(in_mode=IN_PRESCALED,
                       x_in=self.x0s if l == 1 else self.xs[(l - 2) % 2],
                       addend=emb if l == 1 else self.acc,
                       divisor=float(L + 1) if last else 1.0,
                       out=self.acc,
                       xs_out=None if last else self.xs[(l - 1) % 2],
                       **rows)
        if not pruned:
            self._acc_full = self._token(emb)
        return self.acc

    def forward_cached(self, emb: torch.Tensor) -> torch.Tensor:
        """``forward(emb)``, or ``acc`` as it stands when it already holds the
        full layer mean of this table (no update, pruned forward or other
        write since)."""
        if self._acc_full is not None and self._acc_full == self._token(emb):
            return self.acc
        return self.forward(emb)

    def propagate_once(self, x: torch.Tensor, out: torch.Tensor, graph: Graph | None = None):
        """out = Â x (one LGConv call)."""
        self._prop(in_mode=IN_RAW, x_in=x, out=out, graph=graph)

    def propagate_accumulate(self, g_in: torch.Tensor, addend: torch.Tensor,
                             out: torch.Tensor, graph: Graph | None = None):
        """out = Â g_in + addend (generic autograd backward, dense seed)."""
        self._prop(in_mode=IN_RAW, x_in=g_in, addend=addend, out=out, graph=graph)

    # ------------------------------------------------------------------ BPR
    def bpr(self, out: torch.Tensor, emb: torch.Tensor, users, pos, neg, decay: float,
            loss_accum: torch.Tensor | None = None, grad_scale: float = 1.0) -> torch.Tensor:
        """Loss + gradient seeds for one batch of int32 device triples.

        ``grad_scale`` multiplies the gradient seeds (1/world_size under data
        parallelism, so the exchanged seeds / gradients sum to the union
        batch's)."""
        B = int(users.shape[0])
        if B > self.max_batch:
            raise ValueError(f"batch {B} > engine max_batch {self.max_batch}")
        if not self._masks_ready:
            self.compute_frontier(users, pos, neg)  # the seed set S for the backward
        self._ensure_ws(B)
        st = _lib.stream_handle()
        g = self.g
        check(lib.mirec_bpr_forward(out.data_ptr(), emb.data_ptr(), g.n_nodes, g.n_users,
                                    self.dim, B, users.data_ptr(), pos.data_ptr(),
                                    neg.data_ptr(), float(grad_scale), self.coef.data_ptr(),
                                    self.softplus.data_ptr(), self.reg.data_ptr(),
                                    self.keys.data_ptr(), self.vals.data_ptr(), st),
              "bpr_forward")
        check(lib.mirec_bpr_loss(self.softplus.data_ptr(), self.reg.data_ptr(), B,
                                 float(decay), self.loss.data_ptr(), ptr(loss_accum), st),
              "bpr_loss")
        check(lib.mirec_bpr_seed(out.data_ptr(), emb.data_ptr(), g.n_nodes, g.n_users,
                                 self.dim, B, users.data_ptr(), pos.data_ptr(),
                                 neg.data_ptr(), self.coef.data_ptr(), self.keys.data_ptr(),
                                 self.vals.data_ptr(), float(decay), float(grad_scale), self.L,
                                 self.slot.data_ptr(), self.seed_p.data_ptr(),
                                 self.seed_e.data_ptr(), self.keys_sorted.data_ptr(),
                                 self._ws.data_ptr(), self._ws_bytes, st), "bpr_seed")
        self._seeds = (self.seed_p, self.seed_e, self.keys_sorted, 3 * B)
        return self.loss

    # ----------------------------------------------- data-parallel exchange
    def export_seeds(self):
        """Local seeds as fixed-size rows for an all-gather: (keys [3B] int32,
        seed_p [3B, D], seed_e [3B, D]); non-head rows carry key = n_nodes.
        Clears the local slot map (the merged seeds replace it)."""
        seed_p, seed_e, ks, n = self._seeds
        st = _lib.stream_handle()
        packed = self.keys[:n]  # bpr_forward's keys are no longer needed
        check(lib.mirec_seed_pack(ks.data_ptr(), n, self.g.n_nodes, packed.data_ptr(), st),
              "seed_pack")
        check(lib.mirec_bpr_seed_reset(self.slot.data_ptr(), ks.data_ptr(), n, st),
              "bpr_seed_reset")
        self._masks_ready = False
        return packed, seed_p[:n], seed_e[:n]

    def import_seeds(self, keys, rows_p, rows_e):
        """Merge gathered seeds (rank-major order) into this engine's slot map
        and rebuild the frontier of the union seed set."""
        n = int(keys.shape[0])
        if self._merged is None or self._merged[0].shape[0] < n:
            dev, D = self.g.device, self.dim
            self._merged = (torch.empty(n, D, dtype=torch.float32, device=dev),
                            torch.empty(n, D, dtype=torch.float32, device=dev),
                            torch.empty(n, dtype=torch.int32, device=dev))
        mp, me, mk = self._merged
        nb = ctypes.c_size_t(0)
        check(lib.mirec_seed_merge_workspace(n, self.g.n_nodes, ctypes.byref(nb)),
              "seed_merge_workspace")
        if nb.value > self._ws_bytes:
            self._ws = torch.empty(nb.value, dtype=torch.uint8, device=self.g.device)
            self._ws_bytes = nb.value
        check(lib.mirec_seed_merge(keys.data_ptr(), rows_p.data_ptr(), rows_e.data_ptr(), n,
                                   self.dim, self.g.n_nodes, self.slot.data_ptr(), mp.data_ptr(),
                                   me.data_ptr(), mk.data_ptr(), self._ws.data_ptr(),
                                   self._ws_bytes, _lib.stream_handle()), "seed_merge")
        self.compute_frontier(keys=mk, n_keys=n)
        self._seeds = (mp, me, mk, n)

    # ------------------------------------------------------------- backward
    def backward(self, emb: torch.Tensor, adam: AdamState | None = None,
                 grad_out: torch.Tensor | None = None, last_rows=None, on_chunk=None):
        """Horner backward from the current seeds (g_L = d, g_l = d + Â g_{l+1}).

        With ``adam`` the last layer applies Adam to ``emb`` in place (fused);
        otherwise the dense gradient dLoss/dE is written to ``grad_out``.
        ``last_rows`` (static_row_lists) restricts the last layer — and so the
        update — to a fixed row set (a data-parallel rank's shard); the other
        rows of ``emb`` and of the next step's dinv ⊙ E are left alone.  A
        list of row sets runs the last layer as one launch per set, calling
        ``on_chunk(i)`` after launch i (dist.py overlaps the all-gather of
        block i with the launch of block i + 1)."""
        if (adam is None) == (grad_out is None):
            raise ValueError("exactly one of adam / grad_out")
        self._acc_full = None
        if self._seeds is None or not self._masks_ready:
            raise RuntimeError("backward() needs bpr() (or import_seeds()) first")
        L = self.L
        seed_p, seed_e, keys_sorted, n_keys = self._seeds
        hp = adam.next_hparams() if adam is not None else None
        final = dict(seed2=seed_e)
        if adam is not None:
            final.update(adam=(adam, hp), param=emb)
            if L > 0 and self.reuse_prescaled:  # the update also emits the next x~_0
                final.update(xs_out=self.x0s)
        else:
            final.update(out=grad_out)
        chunks = list(last_rows) if isinstance(last_rows, (list, tuple)) else [last_rows]

        def last_layer(**kw):
            for c, rows in enumerate(chunks):
                self._prop(**kw, **final, **(rows or {}))
                if on_chunk is not None:
                    on_chunk(c)
        if L == 0:
            last_layer(in_mode=IN_NONE, seed=seed_p)
        else:
            for l in range(L - 1, -1, -1):
                first = l == L - 1
                if first:
                    # input g_L = d lives on S only; with pruning its output
                    # g_{L-1} is written only on F1 = S ∪ N(S) (zero elsewhere)
                    rows = self._hop_rows() if (self.prune and l > 0) else {}
                    if self.sparse_filter == "dense":
                        kw = dict(in_mode=IN_PRESCALED, x_in=self._dense_seeds(seed_p, 0),
                                  in_mask=self.bm_self, **rows)
                    else:
                        kw = dict(in_mode=IN_SPARSE, seed_in=seed_p,
                                  in_mask=self._sparse_filter(), **rows)
                else:
                    kw = dict(in_mode=IN_PRESCALED, x_in=self.xs[(L - 2 - l) % 2],
                              in_mask=self.bm_hop if (self.prune and l == L - 2) else None)
                kw["seed"] = seed_p
                if l == 0:
                    last_layer(**kw)
                else:
                    kw.update(xs_out=self.xs[(L - 1 - l) % 2])
                    self._prop(**kw)
        if self.sparse_filter == "dense" and L > 0:
            self._dense_seeds(seed_p, 1)
        check(lib.mirec_bpr_seed_reset(self.slot.data_ptr(), keys_sorted.data_ptr(), n_keys,
                                       _lib.stream_handle()), "bpr_seed_reset")
        self._seeds = None
        self._masks_ready = False
        self._x0s_token = self._token(emb) if (adam is not None and L > 0 and last_rows is None
                                               and self.reuse_prescaled) else None

    def adam_step(self, param: torch.Tensor, grad: torch.Tensor, adam: AdamState):
        _note_raw_write()  # the table changes behind its version counter
        self._acc_full = None
        hp = adam.next_hparams()
        check(lib.mirec_adam_dense(param.data_ptr(), grad.data_ptr(), adam.exp_avg.data_ptr(),
                                   adam.exp_avg_sq.data_ptr(), param.numel(), ctypes.byref(hp),
                                   _lib.stream_handle()), "adam_dense")

    # --------------------------------------------------------------- step
    def forward_for_batch(self, emb: torch.Tensor, users, pos, neg) -> torch.Tensor:
        """Frontier of the batch, then the (pruned if enabled) forward."""
        self.compute_frontier(users, pos, neg)
        return self.forward(emb, pruned=self.prune)

    def train_step(self, emb: torch.Tensor, adam: AdamState, users, pos, neg, decay: float,
                   loss_accum: torch.Tensor | None = None) -> torch.Tensor:
        """stageOne: forward, BPR, backward, fused Adam.  Returns loss (device)."""
        out = self.forward_for_batch(emb, users, pos, neg)
        loss = self.bpr(out, emb, users, pos, neg, decay, loss_accum)
        self.backward(emb, adam=adam)
        return loss


def propagate(graph: Graph, x: torch.Tensor, out: torch.Tensor):
    """out = Â x on ``graph`` (one LGConv call; x, out: contiguous fp32
    [n_nodes, D] device tensors, D in SUPPORTED_DIMS)."""
    n, D = x.shape
    if D not in _lib.SUPPORTED_DIMS or n != graph.n_nodes or out.shape != x.shape:
        raise ValueError(f"propagate: x {tuple(x.shape)}, out {tuple(out.shape)}, "
                         f"graph of {graph.n_nodes} nodes")
    if x.dtype != torch.float32 or not (x.is_contiguous() and out.is_contiguous()):
        raise ValueError("propagate: contiguous float32 tensors required")
    p = Prop()
    p.dim = D
    p.in_mode = IN_RAW
    p.x_in = x.data_ptr()
    p.divisor = 1.0
    p.out = out.data_ptr()
    p.partial = ptr(graph.partial_buffer(D))
    p.narrow_max = 64
    check(lib.mirec_propagate(graph.csr_ptr(), ctypes.byref(p), _lib.stream_handle()),
          "propagate")


def sample_triples(graph: Graph, batch: int, seed: int, offset: int, users, pos, neg, err,
                   shard: int = 0, n_shards: int = 1):
    """On-device UniformSample (negative_sample.py:98-134) into int32 buffers
    (the positive weighted by the graph's per-user probabilities when
    ``graph.set_positive_probs`` gave some: negative_sample.py:53-56)."""
    check(lib.mirec_bpr_sample_ex(graph.csr_ptr(), ptr(getattr(graph, "pos_cdf", None)),
                                  graph.n_users, graph.m_items, int(batch),
                                  ctypes.c_uint64(seed & (2**64 - 1)),
                                  ctypes.c_uint64(offset & (2**64 - 1)), int(shard),
                                  int(n_shards), users.data_ptr(), pos.data_ptr(),
                                  neg.data_ptr(), err.data_ptr(), _lib.stream_handle()),
          "bpr_sample")


def sample_epoch_capped(graph: Graph, n_candidates: int, cap: int, seed: int, offset: int = 0,
                        shard: int = 0, n_shards: int = 1, return_candidates: bool = False,
                        n_threads: int | None = None):
    """The ddp_lgcn.py epoch sampler on device (ddp_lgcn.py:33-35, 541-582):
    ``n_candidates`` (= TRAIN_ITERATIVE x trainDataSize) uniform users, a
    positive each, kept while the positive item was kept fewer than ``cap``
    (POSITIVE_NUM_LIMIT) times before in draw order.  Returns int32 device
    (users, pos, neg) of the kept triples in draw order (+ every candidate's
    user and positive, -1 = skipped user, with ``return_candidates``).  A
    graph on the host (a CPU model) runs mirec_cpu_bpr_sample_capped: the same
    streams, the same triples, on ``n_threads`` threads."""
    dev = graph.device
    n = int(n_candidates)
    i32 = dict(dtype=torch.int32, device=dev)
    users, pos, neg = (torch.empty(max(n, 1), **i32) for _ in range(3))
    count = torch.zeros(1, **i32)
    err = torch.zeros(1, **i32)
    cu = torch.empty(max(n, 1), **i32) if return_candidates else None
    cp = torch.empty(max(n, 1), **i32) if return_candidates else None
    if dev.type == "cpu":  # a host model (C1): the same streams on CPU threads
        check(lib.mirec_cpu_bpr_sample_capped(
            graph.rowptr_host.ctypes.data, graph.col_host.ctypes.data, ptr(graph.col_sorted),
            ptr(getattr(graph, "pos_cdf", None)), graph.n_users, graph.m_items, n, int(cap),
            ctypes.c_uint64(seed & (2**64 - 1)), ctypes.c_uint64(offset & (2**64 - 1)),
            int(shard), int(n_shards), users.data_ptr(), pos.data_ptr(), neg.data_ptr(),
            count.data_ptr(), err.data_ptr(), ptr(cu), ptr(cp),
            int(n_threads or os.cpu_count() or 1)), "cpu_bpr_sample_capped")
        k = int(count.item())
        if int(err.item()) != 0:
            raise RuntimeError("sampler: a user has every item as a positive")
        out = (users[:k], pos[:k], neg[:k])
        return out + (cu[:n], cp[:n]) if return_candidates else out
    nb = ctypes.c_size_t(0)
    check(lib.mirec_bpr_sample_capped_workspace(n, graph.m_items, ctypes.byref(nb)),
          "bpr_sample_capped_workspace")
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
    check(lib.mirec_bpr_sample_capped_ex(graph.csr_ptr(), ptr(getattr(graph, "pos_cdf", None)),
                                         graph.n_users, graph.m_items, n, int(cap),
                                         ctypes.c_uint64(seed & (2**64 - 1)),
                                         ctypes.c_uint64(offset & (2**64 - 1)), int(shard),
                                         int(n_shards), users.data_ptr(), pos.data_ptr(),
                                         neg.data_ptr(), count.data_ptr(), err.data_ptr(),
                                         ptr(cu), ptr(cp), ws.data_ptr(), nb.value,
                                         _lib.stream_handle()),
          "bpr_sample_capped")
    k = int(count.item())
    if int(err.item()) != 0:
        raise RuntimeError("sampler: a user has every item as a positive")
    out = (users[:k], pos[:k], neg[:k])
    return out + (cu[:n], cp[:n]) if return_candidates else out


_ = math
