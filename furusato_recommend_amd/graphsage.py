"""GraphSAGE (model/graphsage.py:31-477) on the HIP engine — the hop path.

In scope: on-device fixed-fanout neighbour sampling and
the per-hop aggregation h = W_i · [x_target ; mean_j dropout(x_j)] (+ReLU
except the last layer, graphsage.py:311-324), the BPR loss with the
reference's parameter-norm term (:326-337), OneEpoch (:339-399) and the
full-graph inference of getUsersRating('all') (:401-424).
Out of scope: the proprietary feature / text towers feeding the initial
embedding (:135-161, 163-303) — the initial node embedding here is the id
embedding alone, so the first layer is Linear(2d -> d) instead of the
reference's Linear(4d -> d) over [id ; feature] embeddings.

Sampling tree.  PyG's NeighborSampler (graphsage.py:342-365) samples hop h
for every node already in the batch, without replacement (all neighbours
when the degree is at most the fanout); here every tree slot draws its own
children — a node reached twice gets two independent draws where PyG
samples a deduplicated node once, the same distribution per occurrence —
and a fixed fanout with -1 in the slots a short row cannot fill makes the
structure a regular tree of node groups (``fanout_replace=True`` draws with
replacement, as the repo's uniform_neighbors, neighbor_sampling.py:14-30,
except that a node without neighbours gets no children — mean 0, PyG's
behaviour — where uniform_neighbors draws random ids): every node at depth d gets
a child group for each hop h = d+1..L (sizes[h-1] children each), and layer
i (hop L-i) updates every group of depth <= L-1-i from its hop-(L-i)
children.  All groups' rows are gathered from the embedding table in ONE
launch (mirec_gather_rows; backward = one atomic scatter-add), every hop mean
is one mirec_fanout_mean (dropout fused, mask recomputed in the backward),
the Linear layers run on f32 MFMA GEMMs (csrc/gemm.hip via linear.py).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import engine as _engine
from ._lib import CSR, IN_PRESCALED, Prop, check, lib
from .engine import AdamGroup, AdamState, sample_triples
from .graph import DEFAULT_SPLIT, Graph, positive_probs
from .linear import Linear, sage_linear
from .rows import slice_norms2


# The id table's backward: the deterministic sorted form (True: every row
# contribution of the tree sorted by row id and summed in entry order, Adam
# fused on top, no dense gradient written) or the float-atomic scatter into a
# dense gradient (False; A/B timing, tools/bench_sage.py --leaf-bwd atomic).
SORTED_LEAF_BACKWARD = True


def _BWD_ON_CALLER():
    """The step's backward runs on the calling thread instead of autograd's
    device thread: the same launches on the same stream, without the
    hand-off (a micro-batch's backward issue took 0.43 ms of host through the
    device thread, 0.25 ms on the caller; profiles/round4_host_profile_sage_*)."""
    return torch.autograd.set_multithreading_enabled(False)


class TableGrad:
    """The table gradient of one step in the sorted form (csrc/tablegrad.hip):
    G = c[slice] * table + S, with S stored in ``acc`` for the rows whose
    ``stamp`` equals ``gen`` (never cleared) and c = (c_user, c_item) the
    norm-term coefficients on the device.  ``dense`` selects whether the
    backward also materialises G as the table's .grad (data parallelism,
    which all-reduces it) or leaves it to ``adam`` (single GPU)."""

    def __init__(self, n_rows: int, n_user: int, dim: int, device):
        self.n_rows, self.n_user, self.dim = int(n_rows), int(n_user), int(dim)
        self.acc = torch.empty(n_rows, dim, device=device)
        self.stamp = torch.zeros(n_rows, dtype=torch.int32, device=device)
        self.coef = torch.zeros(2, device=device)
        self.gen = 0
        self.pending = False  # S / coef of the last backward not yet consumed
        self.adam_events = None  # a list: (start, end) HIP events of each adam()
        self.dense = False
        # static: a HIP-graph-captured step bakes the generation into its
        # launches, so every step clears the stamps and reuses generation 1
        self.static = False
        # atomic: S by float atomics (plain groups only; no sort, order of a
        # repeated id's sum not fixed) instead of the sorted segmented sums
        self.atomic = False
        self._ws = None
        self.entries = 0  # row contributions of the last accumulate
        # packed export (the pipelined data-parallel exchange): with rows_parts
        # = P the accumulate writes S packed — (rows ascending, vals, counts
        # [1 + P] per owner block), mirec_table_grad_sorted_rows — into
        # ``export`` instead of acc / stamp (nothing stamped: a dense consumer
        # sees S = 0, never stale rows)
        self.rows_parts = None
        self.export = None

    def accumulate(self, groups):
        """groups: [(ids int32, grad_out [n_t, d], k, mean, dropout p, seed)]."""
        n = len(groups)
        if not 1 <= n <= _lib.TABLE_GRAD_MAX_GROUPS:
            raise ValueError("table gradient: 1..8 row groups")
        self.entries = sum(int(g[0].numel()) for g in groups)  # bounds the rows stamped
        arr = (_lib.RowGradGroup * n)()
        keep = []
        for a, (ids, g, k, mean, p, seed) in zip(arr, groups):
            g = g.contiguous()
            keep.append(g)
            a.ids, a.grad_out = ids.data_ptr(), g.data_ptr()
            a.n_targets, a.k, a.mean = ids.numel() // k, int(k), int(mean)
            a.dropout_p, a.seed = float(p), int(seed)
        if self.atomic:
            self._next_gen()
            check(lib.mirec_table_grad_atomic(arr, n, self.n_rows, self.dim, self.acc.data_ptr(),
                                              self.stamp.data_ptr(), self.gen,
                                              _lib.stream_handle()), "table_grad_atomic")
            self.pending = True
            return
        nb = ctypes.c_size_t()
        check(lib.mirec_table_grad_workspace(arr, n, self.n_rows, self.dim, ctypes.byref(nb)),
              "table_grad_workspace")
        if self._ws is None or self._ws.numel() < nb.value:
            self._ws = torch.empty(nb.value, dtype=torch.uint8, device=self.acc.device)
        self._next_gen()
        if self.rows_parts:
            dev = self.acc.device
            cap = max(min(self.n_rows, self.entries), 1)
            rows = torch.empty(cap, dtype=torch.int32, device=dev)
            vals = torch.empty(cap, self.dim, device=dev)
            counts = torch.empty(1 + int(self.rows_parts), dtype=torch.int32, device=dev)
            check(lib.mirec_table_grad_sorted_rows(arr, n, self.n_rows, self.dim,
                                                   int(self.rows_parts), rows.data_ptr(),
                                                   vals.data_ptr(), counts.data_ptr(),
                                                   self._ws.data_ptr(), self._ws.numel(),
                                                   _lib.stream_handle()), "table_grad_sorted_rows")
            self.export = (rows, vals, counts)
            self.pending = True
            return
        check(lib.mirec_table_grad_sorted(arr, n, self.n_rows, self.dim, self.acc.data_ptr(),
                                          self.stamp.data_ptr(), self.gen, self._ws.data_ptr(),
                                          self._ws.numel(), _lib.stream_handle()),
              "table_grad_sorted")
        self.pending = True

    def _next_gen(self):
        if self.static:
            self.stamp.zero_()
            self.gen = 1
        else:
            self.gen += 1

    def skip(self):
        """A backward with no row gradient: S = 0 (a fresh generation)."""
        self._next_gen()
        self.entries = 0
        self.export = None
        self.pending = True

    def materialize(self, table: torch.Tensor) -> torch.Tensor:
        """G as a dense [N, d] tensor."""
        grad = torch.empty_like(table)
        check(lib.mirec_table_grad_dense(table.data_ptr(), self.coef.data_ptr(), self.n_user,
                                         self.acc.data_ptr(), self.stamp.data_ptr(), self.gen,
                                         self.n_rows, self.dim, grad.data_ptr(),
                                         _lib.stream_handle()), "table_grad_dense")
        return grad

    def adam(self, state: AdamState, norms: torch.Tensor | None = None,
             h_dev: torch.Tensor | None = None):
        """One Adam step of the table with G formed in the kernel; writes the
        updated slices' norms to ``norms`` (2 floats) if given.  With
        ``h_dev`` the hyper-parameters are read from that device buffer when
        the kernel runs (a captured step; the host step count is not
        advanced)."""
        sumsq = None
        if norms is not None:
            sumsq = torch.empty(int(lib.mirec_adam_table_sumsq_floats(self.n_rows, self.dim)),
                                device=self.acc.device)
        args = (state.param.data_ptr(), state.exp_avg.data_ptr(), state.exp_avg_sq.data_ptr(),
                self.coef.data_ptr(), self.n_user, self.acc.data_ptr(), self.stamp.data_ptr(),
                self.gen, self.n_rows, self.dim)
        ev = self.adam_events  # bench: HIP events around the launch (its stream)
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if h_dev is None:
            hp = state.next_hparams()
            check(lib.mirec_adam_table(*args, ctypes.byref(hp), _lib.ptr(sumsq), _lib.ptr(norms),
                                       _lib.stream_handle()), "adam_table")
        else:
            check(lib.mirec_adam_table_dev(*args, h_dev.data_ptr(), _lib.ptr(sumsq),
                                           _lib.ptr(norms), _lib.stream_handle()),
                  "adam_table_dev")
        if ev is not None:
            e1.record()
            ev.append((e0, e1))
        _engine._note_raw_write()
        self.pending = False


# ----------------------------------------------------------------- autograd
class _TableTerms(torch.autograd.Function):
    """Everything the loss takes from the [N, d] id table in one node:
      * rows = table[ids] for the tree's inner groups (their raw rows feed
        layer 0 as self features),
      * for every leaf group (depth L: only ever averaged by its parent at
        layer 0) the parent's dropout-mean over its children's table rows,
        gathered and averaged in one pass (mirec_fanout_mean_gather) — the
        leaf rows, ~90 % of a [25, 10] tree, are never materialised,
      * the norms of the user and item slices (graphsage.py:326-337; reused
        from the previous step's fused Adam when the table is unchanged).
    Backward, sorted form (``sink`` given): the inner row gradients and every
    leaf entry's mask * g_out[t] / cnt_t are sorted by row id and summed in
    entry order (mirec_table_grad_sorted) and the norm coefficients are kept
    on the device — the dense gradient is formed inside the Adam kernel, or
    materialised for data parallelism.  Atomic form (``sink`` None): the
    dense gradient [g_u u/|u| ; g_i i/|i|] is written, then the row
    gradients are scatter-added with float atomics.
    ``leaves`` = ((ids, k, dropout p, seed), ...)."""

    @staticmethod
    def forward(ctx, table, ids, n_user: int, leaves, sink, norms, splits):
        n, d = ids.numel(), table.shape[1]
        st = _lib.stream_handle()
        rows = torch.empty(n, d, dtype=table.dtype, device=table.device)
        check(lib.mirec_gather_rows(table.data_ptr(), ids.data_ptr(), n, d, rows.data_ptr(), st),
              "gather_rows")
        aggrs = []
        for lid, k, p, seed in leaves:
            n_t = lid.numel() // k
            out = torch.empty(n_t, d, dtype=table.dtype, device=table.device)
            check(lib.mirec_fanout_mean_gather(table.data_ptr(), lid.data_ptr(), n_t, k, d,
                                               float(p), ctypes.c_uint64(seed), out.data_ptr(),
                                               st), "fanout_mean_gather")
            aggrs.append(out)
        # both slices' norms in one pass (or the previous step's fused Adam's,
        # read in place: the next Adam rewrites it only after this backward)
        norms2 = slice_norms2(table, n_user) if norms is None else norms.view(2)
        ctx.save_for_backward(table, ids, norms2, *[l[0] for l in leaves])
        ctx.leaf_cfg = [(k, p, seed) for _, k, p, seed in leaves]
        ctx.n_user = n_user
        ctx.sink = sink
        ctx.splits = tuple(int(x) for x in splits)
        ctx.set_materialize_grads(False)
        # the inner groups' rows as separate outputs: their gradients arrive
        # separately (no concatenation) and become separate row groups
        return (*rows.split(ctx.splits), norms2, *aggrs)

    @staticmethod
    def backward(ctx, *grads):
        P = len(ctx.splits)
        g_parts, g_norms, g_aggrs = grads[:P], grads[P], grads[P + 1:]
        table, ids, norms2, *leaf_ids = ctx.saved_tensors
        id_parts = ids.split(ctx.splits)
        k = ctx.n_user
        d = table.shape[1]
        st = _lib.stream_handle()
        # d|x|/dx = x/|x| (0 for a zero slice, as torch's norm backward)
        sink = ctx.sink
        if sink is not None:
            if g_norms is None:
                sink.coef.zero_()
            else:
                check(lib.mirec_norm_coef(g_norms.contiguous().data_ptr(), 1, norms2.data_ptr(), 1,
                                          2, sink.coef.data_ptr(), st), "norm_coef")
            groups = [(i, g, 1, 0, 0.0, 0) for i, g in zip(id_parts, g_parts)
                      if g is not None and i.numel() > 0]
            for g, lid, (kk, p, seed) in zip(g_aggrs, leaf_ids, ctx.leaf_cfg):
                if g is not None:
                    groups.append((lid, g, kk, 1, p, seed))
            if groups:
                sink.accumulate(groups)
            else:  # S = 0: a fresh generation stamps nothing
                sink.skip()
            return (sink.materialize(table) if sink.dense else None), None, None, None, None, None, \
                None
        if g_norms is None:
            coef = torch.zeros_like(norms2)
        else:
            coef = torch.where(norms2 > 0, g_norms / norms2, torch.zeros_like(norms2))
        cu, ci = coef[0], coef[1]
        grad = torch.empty_like(table)
        torch.mul(table[:k], cu, out=grad[:k])
        torch.mul(table[k:], ci, out=grad[k:])
        for i, g in zip(id_parts, g_parts):
            if g is not None and i.numel() > 0:
                check(lib.mirec_scatter_add_rows(g.contiguous().data_ptr(), i.data_ptr(),
                                                 i.numel(), d, grad.data_ptr(), st),
                      "scatter_add_rows")
        for g, lid, (kk, p, seed) in zip(g_aggrs, leaf_ids, ctx.leaf_cfg):
            if g is None:
                continue
            n_t = lid.numel() // kk
            check(lib.mirec_fanout_mean_gather_bwd(g.contiguous().data_ptr(), lid.data_ptr(),
                                                   n_t, kk, d, float(p), ctypes.c_uint64(seed),
                                                   grad.data_ptr(), st),
                  "fanout_mean_gather_bwd")
        return grad, None, None, None, None, None, None


class _SageLoss(torch.autograd.Function):
    """The GraphSAGE BPR loss (model/graphsage.py:326-337) in two launches:
    mean softplus(<u,n> - <u,p>) over the seed embeddings out3 = [u ; p ; n]
    plus decay / B * all_param, where the reference's doubling accumulation
    all_param = 2 all_param + |p_k| over (user ids, item ids, w_0, b_0, ...)
    is the weighted sum Σ_k 2^(K-1-k) |p_k| (mirec_norm_terms: the table
    slices' norms come in as ``norms2``, the small parameters' are computed
    in the same launch), then mirec_bpr_rows_loss.  Backward: the row
    gradients of out3 in one buffer, the small parameters' gradients and the
    table slices' norm gradients in one launch."""

    @staticmethod
    def forward(ctx, out3, norms2, decay: float, *small):
        B = out3.shape[0] // 3
        d = out3.shape[1]
        K = 2 + len(small)
        st = _lib.stream_handle()
        dev = out3.device
        w_small = [float(2 ** (K - 3 - k)) for k in range(len(small))]
        w_extra = [float(2 ** (K - 1)), float(2 ** (K - 2))]
        xs = (ctypes.c_void_p * max(1, len(small)))(*[t.data_ptr() for t in small])
        numel = (ctypes.c_int64 * max(1, len(small)))(*[t.numel() for t in small])
        wk = (ctypes.c_float * max(1, len(small)))(*w_small)
        we = (ctypes.c_float * 2)(*w_extra)
        norms = torch.empty(max(1, len(small)), device=dev)
        total = torch.empty(1, device=dev)
        check(lib.mirec_norm_terms(xs, numel, wk, len(small), norms2.data_ptr(), we, 2,
                                   norms.data_ptr(), total.data_ptr(), st), "norm_terms")
        x = torch.empty(2 * B, device=dev)
        loss = torch.empty(1, device=dev)
        coef = float(decay) / B
        check(lib.mirec_bpr_rows_loss(out3.data_ptr(), out3[B:].data_ptr(),
                                      out3[2 * B:].data_ptr(), B, d, total.data_ptr(), coef,
                                      x.data_ptr(), loss.data_ptr(), st), "bpr_rows_loss")
        ctx.save_for_backward(out3, x, norms, *small)
        ctx.cfg = (B, d, coef, w_small, w_extra)
        ctx.small_params = small  # the leaf Parameters (their .grad gets the norm term)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        out3, x, norms, *small = ctx.saved_tensors
        B, d, coef, w_small, w_extra = ctx.cfg
        st = _lib.stream_handle()
        g = g.reshape(1).contiguous()
        d_out3 = torch.empty_like(out3)
        g_extra = torch.empty(1, device=out3.device)
        check(lib.mirec_bpr_rows_loss_bwd(out3.data_ptr(), out3[B:].data_ptr(),
                                          out3[2 * B:].data_ptr(), x.data_ptr(), B, d,
                                          g.data_ptr(), coef, d_out3.data_ptr(),
                                          d_out3[B:].data_ptr(), d_out3[2 * B:].data_ptr(),
                                          g_extra.data_ptr(), st), "bpr_rows_loss_bwd")
        we = (ctypes.c_float * 2)(*w_extra)
        g_norms2 = torch.empty(2, device=out3.device)
        check(lib.mirec_norm_terms_bwd(None, None, None, None, 0, None, g_extra.data_ptr(), we, 2,
                                       g_norms2.data_ptr(), st), "norm_terms_bwd")
        if not small:
            return (d_out3, g_norms2, None)
        # The small parameters' norm gradients are ADDED to their .grad once
        # the whole backward has run (each Linear parameter also gets its
        # GEMM gradient, the first layer's twice): one launch instead of an
        # elementwise add per extra use.
        params = ctx.small_params

        def add_norm_grads():
            for p in params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            n = len(params)
            xs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in small])
            gs = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in params])
            numel = (ctypes.c_int64 * n)(*[t.numel() for t in small])
            wk = (ctypes.c_float * n)(*w_small)
            check(lib.mirec_norm_terms_bwd_acc(xs, gs, numel, wk, n, norms.data_ptr(),
                                               g_extra.data_ptr(), _lib.stream_handle()),
                  "norm_terms_bwd_acc")

        torch.autograd.Variable._execution_engine.queue_callback(add_norm_grads)
        return (d_out3, g_norms2, None, *[None] * len(small))


class _FanoutMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, valid, k, p, seed):
        n_t = valid.numel() // k
        d = x.shape[1]
        out = torch.empty(n_t, d, dtype=x.dtype, device=x.device)
        check(lib.mirec_fanout_mean(x.contiguous().data_ptr(), valid.data_ptr(), n_t, k, d,
                                    float(p), ctypes.c_uint64(seed), out.data_ptr(),
                                    _lib.stream_handle()), "fanout_mean")
        ctx.save_for_backward(valid)
        ctx.cfg = (n_t, k, d, float(p), seed)
        return out

    @staticmethod
    def backward(ctx, grad):
        (valid,) = ctx.saved_tensors
        n_t, k, d, p, seed = ctx.cfg
        gx = torch.empty(n_t * k, d, dtype=grad.dtype, device=grad.device)
        check(lib.mirec_fanout_mean_bwd(grad.contiguous().data_ptr(), valid.data_ptr(), n_t, k,
                                        d, p, ctypes.c_uint64(seed), gx.data_ptr(),
                                        _lib.stream_handle()), "fanout_mean_bwd")
        return gx, None, None, None, None


def csr_mean(graph: Graph, mean_dinv: torch.Tensor, x: torch.Tensor, out: torch.Tensor):
    """out_i = mean_{j in N(i)} x_j (0 for isolated i): the CSR propagation
    kernel with row scale 1/deg_i and un-scaled inputs (graphsage.py:411-416)."""
    c = CSR.from_buffer_copy(graph.csr)
    c.dinv = mean_dinv.data_ptr()
    p = Prop()
    p.dim = x.shape[1]
    p.in_mode = IN_PRESCALED
    p.x_in = x.data_ptr()
    p.divisor = 1.0
    p.out = out.data_ptr()
    p.partial = _lib.ptr(graph.partial_buffer(x.shape[1]))
    p.narrow_max = 64
    check(lib.mirec_propagate(ctypes.byref(c), ctypes.byref(p), _lib.stream_handle()),
          "propagate(mean)")


# -------------------------------------------------------------------- model
class SampleTree:
    """Node groups of a fixed-fanout sampled tree (see module docstring)."""

    def __init__(self):
        self.groups = []       # [ids (int32, -1 = none), depth]
        self.children = {}     # (group index, hop) -> child group index

    def add(self, ids, depth):
        self.groups.append((ids, depth))
        return len(self.groups) - 1

    @staticmethod
    def canonical_layout(L: int):
        """(depths, children) of the group order sample_tree produces."""
        depths, children = [0], {}

        def expand(gi):
            for h in range(depths[gi] + 1, L + 1):
                depths.append(h)
                ci = len(depths) - 1
                children[(gi, h)] = ci
                expand(ci)

        expand(0)
        return depths, children

    @classmethod
    def from_groups(cls, groups, L: int):
        """Tree from explicit per-group id tensors in canonical order."""
        depths, children = cls.canonical_layout(L)
        if len(groups) != len(depths):
            raise ValueError("group count does not match the canonical layout")
        t = cls()
        t.groups = [(g, d) for g, d in zip(groups, depths)]
        t.children = children
        return t


class _ChunkTrees:
    """The C micro-batch trees of a step as a sequence whose tree k is
    sampled when first accessed (trees before it first)."""

    def __init__(self, sample, C: int):
        self._sample = sample
        self._trees = [None] * C

    def __len__(self):
        return len(self._trees)

    def __getitem__(self, k: int):
        n = len(self._trees)
        if k < 0:
            k += n
        if not 0 <= k < n:
            raise IndexError(f"micro-batch tree {k} of {n}")
        for j in range(k + 1):
            if self._trees[j] is None:
                self._trees[j] = self._sample(j)
        return self._trees[k]

    def __iter__(self):
        return (self[k] for k in range(len(self)))


class GraphSAGE(nn.Module):
    def __init__(self, config: dict, dataset):
        super().__init__()
        self.config = config
        self.n_user = self.num_users = int(dataset.n_users)
        self.m_item = self.num_items = int(dataset.m_items)
        self.latent_dim = d = int(config.get("recdim", 128))
        self.num_layers = L = int(config.get("layer", 2))
        k = int(config.get("num_neighbors", 5))
        self.sizes = [int(s) for s in config.get("fanouts", [k] * L)]
        if len(self.sizes) != L:
            raise ValueError("fanouts must have one size per layer")
        self.dropout_p = float(config.get("dropout_p", 0.2))
        # neighbour sampling: without replacement (False, default: PyG's
        # NeighborSampler of graphsage.py:342-365 — all neighbours when the
        # degree is <= the fanout) or with replacement (True: the repo's
        # uniform_neighbors, neighbor_sampling.py:14-30)
        self.fanout_replace = bool(config.get("fanout_replace", False))
        self.device = torch.device(config.get("device", "cuda:0"))
        if self.device.type != "cuda":
            raise RuntimeError("GraphSAGE (furusato_recommend_amd) runs on a HIP device only")
        if d % 4 != 0:
            raise ValueError("recdim must be a multiple of 4")
        n = self.n_user + self.m_item
        # one [N, d] table; the reference's two id tables are views into it
        self._table = nn.Parameter(torch.empty(n, d, device=self.device))
        self.w_linears = nn.ModuleList(
            [Linear(2 * d, d, device=self.device) for _ in range(L)])
        self.init_parameters()
        self.graph = Graph.from_interactions(dataset.trainUser, dataset.trainItem,
                                             self.n_user, self.m_item, self.device,
                                             split=int(config.get("csr_split", DEFAULT_SPLIT)))
        self.graph.set_positive_probs(positive_probs(config))
        deg = torch.from_numpy(self.graph.degree()).to(self.device).float()
        self._mean_dinv = torch.where(deg > 0, 1.0 / deg.clamp(min=1), torch.zeros_like(deg))
        # the table's Adam state is stepped by the fused kernel (TableGrad.adam)
        # or, when its gradient is materialised, with the others
        self._table_state = AdamState(self._table, lr=config["lr"])
        self.optims = AdamGroup([self._table_state] +
                                [AdamState(p, lr=config["lr"]) for p in self.w_linears.parameters()])
        self._tg = TableGrad(n, self.n_user, d, self.device)
        self._norm_cache = None  # (norms [2], token) of the table after the fused Adam
        self._step_seed = int(config.get("seed", 2020))
        self._calls = 0
        # set by DenseGradDataParallel's ``fetch`` exchange: the local table
        # is current on this rank's row block and the fetched rows only
        # until sync_table() / gather_optimizer_state() (collectives) run
        self.table_stale = False
        self.register_state_dict_pre_hook(
            lambda module, prefix, keep_vars: module._check_table_current("state_dict()"))

    def _check_table_current(self, what: str):
        if self.table_stale:
            raise RuntimeError(f"GraphSAGE.{what}: the id table is current on this rank's row "
                               "block only (data-parallel 'fetch' exchange); call "
                               "sync_table() or gather_optimizer_state() on every rank first")

    @property
    def user_id_embeddings(self):
        return self._table[: self.n_user]

    @property
    def item_id_embeddings(self):
        return self._table[self.n_user:]

    def init_parameters(self):
        # graphsage.py:123-133 (gain 0.1; the last w_linear at gain 1)
        gain = 0.1
        with torch.no_grad():
            nn.init.normal_(self._table, std=gain)
            for i, w in enumerate(self.w_linears):
                nn.init.xavier_uniform_(w.weight, gain=1.0 if i == self.num_layers - 1 else gain)
                nn.init.zeros_(w.bias)

    # ------------------------------------------------------------ sampling
    def sample_tree(self, seeds: torch.Tensor, seed: int) -> SampleTree:
        L = self.num_layers
        tree = SampleTree()
        root = tree.add(seeds.to(torch.int32).contiguous(), 0)
        offset = 0

        def expand(gi):
            nonlocal offset
            ids, depth = tree.groups[gi]
            for h in range(depth + 1, L + 1):
                k = self.sizes[h - 1]
                ch = torch.empty(ids.numel() * k, dtype=torch.int32, device=self.device)
                fn = lib.mirec_sample_fanout if self.fanout_replace else \
                    lib.mirec_sample_fanout_norep
                check(fn(self.graph.csr_ptr(), ids.data_ptr(), ids.numel(), k,
                         ctypes.c_uint64(seed), ctypes.c_uint64(offset), ch.data_ptr(),
                         _lib.stream_handle()), "sample_fanout")
                offset += ch.numel()
                ci = tree.add(ch, h)
                tree.children[(gi, h)] = ci
                expand(ci)

        expand(root)
        return tree

    # ------------------------------------------------------------- forward
    def forward(self, tree: SampleTree, dropout_seed: int | None = None) -> torch.Tensor:
        """Seed embeddings h^(L) for a sampled tree (graphsage.py:311-324)."""
        L = self.num_layers
        p = self.dropout_p if (self.training and dropout_seed is not None) else 0.0
        groups = tree.groups
        parent = {ci: gi for (gi, _), ci in tree.children.items()}

        def seed_of(gi, i):
            return 0 if p == 0.0 else (dropout_seed * 1_000_003 + gi * 131 + i)

        # leaves (depth L) are only averaged by their parents at layer 0:
        # fused gather + mean inside the table node
        inner = [gi for gi, (_, dep) in enumerate(groups) if dep < L]
        leaf = [ci for ci, (_, dep) in enumerate(groups) if dep == L]
        leaves = tuple((groups[ci][0], self.sizes[L - 1], p, seed_of(parent[ci], 0))
                       for ci in leaf)
        ids = torch.cat([groups[gi][0] for gi in inner])
        sink = self._tg if SORTED_LEAF_BACKWARD else None
        splits = [groups[gi][0].numel() for gi in inner]
        out = _TableTerms.apply(self._table, ids, self.n_user, leaves, sink,
                                self._cached_norms(), splits)
        parts, norms2, aggrs = out[:len(inner)], out[len(inner)], out[len(inner) + 1:]
        self._slice_norms2 = norms2  # consumed by loss() / the fused loss
        # one output per inner group (the table node's backward takes their
        # gradients as separate row groups)
        h = [None] * len(groups)
        for gi, part in zip(inner, parts):
            h[gi] = part
        leaf_aggr = {parent[ci]: a for ci, a in zip(leaf, aggrs)}
        for i in range(L):
            hop = L - i
            new = list(h)
            for gi, (g, depth) in enumerate(groups):
                if depth > L - 1 - i:
                    continue
                ci = tree.children[(gi, hop)]
                k = self.sizes[hop - 1]
                if i == 0:
                    aggr = leaf_aggr[gi]  # children at hop L are leaves
                else:
                    aggr = _FanoutMean.apply(h[ci], groups[ci][0], k, p, seed_of(gi, i))
                lin = self.w_linears[i]
                new[gi] = sage_linear(h[gi], aggr, lin.weight, lin.bias, relu=i != L - 1)
            h = new
        return h[0]

    def table_grad_dense(self) -> torch.Tensor:
        """The id table's gradient after a backward (before the step), as a
        dense [N, d] tensor."""
        if self._table.grad is not None:
            return self._table.grad
        if not self._tg.pending:
            raise RuntimeError("no pending table gradient")
        return self._tg.materialize(self._table.detach())

    def _norm_token(self):
        return (self._table._version, _engine._raw_writes)

    def _cached_norms(self):
        c = self._norm_cache
        if c is not None and c[1] == self._norm_token():
            return c[0]
        self._norm_cache = None
        return None

    @torch.no_grad()
    def optimizer_step(self):
        """Adam over every parameter (graphsage.py:388-397): the Linear
        layers with the multi-tensor kernel; the table through the fused
        kernel from the pending sorted gradient (which also leaves the
        updated slices' norms for the next forward), or with the others when
        its gradient was materialised."""
        if self._table.grad is not None or not self._tg.pending:
            self.optims.step()
            self._tg.pending = False
            return
        lin = AdamGroup(self.optims.states[1:])
        lin.step()
        norms = torch.empty(2, device=self.device)
        self._tg.adam(self._table_state, norms)
        _engine._note_raw_write()
        self._norm_cache = (norms, self._norm_token())

    def reg_parameters(self):
        """The in-scope parameters in the reference's registration order
        (graphsage.py:96-118): user ids, item ids, then w_linears."""
        out = [self._table[: self.n_user], self._table[self.n_user:]]
        for w in self.w_linears:
            out += [w.weight, w.bias]
        return out

    def loss(self, user_emb, pos_emb, neg_emb, decay_scale: float = 1.0):
        """graphsage.py:326-337, including its parameter-norm accumulation
        (all_param += all_param + |p|, i.e. doubling) over the parameters.
        ``decay_scale`` scales the norm term (1/C for each of C micro-batches
        of one batch, so their summed gradients are the batch's)."""
        pos_scores = torch.sum(user_emb * pos_emb, dim=1)
        neg_scores = torch.sum(user_emb * neg_emb, dim=1)
        all_param = 0
        n2 = getattr(self, "_slice_norms2", None)
        self._slice_norms2 = None
        norms = None if n2 is None else (n2[0], n2[1])
        for k, prm in enumerate(self.reg_parameters()):
            # the two table slices' norms come from the forward's fused node
            nrm = norms[k] if (k < 2 and norms is not None) else prm.norm(2)
            all_param = all_param + all_param + nrm
        all_param = all_param / user_emb.size(0)
        loss = torch.mean(F.softplus(neg_scores - pos_scores))
        return loss + all_param * (self.config["decay"] * decay_scale)

    def loss_fused(self, emb: torch.Tensor, decay_scale: float = 1.0) -> torch.Tensor:
        """loss() on the forward's seed embeddings emb = [u ; p ; n] [3B, d]
        in two launches (_SageLoss); the same value up to fp32 order."""
        n2 = getattr(self, "_slice_norms2", None)
        if n2 is None or not emb.is_contiguous() or emb.shape[1] % 4:
            B = emb.shape[0] // 3
            return self.loss(emb[:B], emb[B:2 * B], emb[2 * B:], decay_scale)
        self._slice_norms2 = None
        small = [q for w in self.w_linears for q in (w.weight, w.bias)]
        return _SageLoss.apply(emb, n2, float(self.config["decay"]) * decay_scale, *small)

    def embed_triples(self, users, pos, neg, seed: int):
        """One tree over the 3B seeds (users, pos+n_user, neg+n_user)."""
        B = users.numel()
        seeds = torch.cat([users.int(), pos.int() + self.n_user, neg.int() + self.n_user])
        tree = self.sample_tree(seeds.to(self.device), seed)
        emb = self.forward(tree, dropout_seed=seed if self.training else None)
        return emb[:B], emb[B: 2 * B], emb[2 * B:]

    # ------------------------------------------------------------ training
    def stageOne(self, users, pos, neg, grad_hook=None, loss_scale: float = 1.0,
                 tree: SampleTree | None = None, tree_hook=None, chunks: int = 1,
                 chunk_hook=None):
        """One BPR step (graphsage.py:366-397).  ``loss_scale`` scales the
        gradient (1/world_size under data parallelism); ``grad_hook`` runs
        between backward and Adam (the gradient all-reduce); ``tree_hook(tree)``
        runs between sampling and the forward (DenseGradDataParallel's row
        fetch).  ``chunks`` = C > 1 (with ``chunk_hook``, the pipelined fetch
        exchange): the batch as C micro-batches of its triples, one tree each
        (``chunk_seeds``; ``tree_hook`` gets them as a sequence whose tree k
        is sampled when the hook first reaches it), then per micro-batch ``chunk_hook(k, "pre")``, forward, loss
        weighted so the micro-batches' gradients sum to the batch's
        (``_stage_chunks``), backward, ``chunk_hook(k, "post")`` — the hook exports each
        micro-batch's table-gradient rows before the next overwrites them."""
        seed = self._step_seed * 7919 + self._calls
        self._calls += 1
        for p in self.parameters():
            p.grad = None
        if chunks > 1:
            if chunk_hook is None or tree is not None:
                raise ValueError("micro-batched steps need a chunk_hook (DP fetch exchange)")
            return self._stage_chunks(users, pos, neg, seed, grad_hook, loss_scale, tree_hook,
                                      int(chunks), chunk_hook)
        if tree is None:
            u32, p32, n32 = (torch.as_tensor(t).to(device=self.device, dtype=torch.int32)
                             .contiguous() for t in (users, pos, neg))
            seeds = torch.empty(3 * u32.numel(), dtype=torch.int32, device=u32.device)
            check(lib.mirec_pack_seed_nodes(u32.data_ptr(), p32.data_ptr(), n32.data_ptr(),
                                            u32.numel(), self.n_user, seeds.data_ptr(),
                                            _lib.stream_handle()), "pack_seed_nodes")
            tree = self.sample_tree(seeds, seed)
        if tree_hook is not None:
            tree_hook(tree)
        emb = self.forward(tree, dropout_seed=seed if self.training else None)
        loss = self.loss_fused(emb)
        one = self.__dict__.get("_loss_seed")  # kept: no fill kernel per step
        if one is None or one.device != loss.device:
            one = self._loss_seed = torch.ones((), dtype=loss.dtype, device=loss.device)
        with _BWD_ON_CALLER():
            loss.backward(one if loss_scale == 1.0 else one * loss_scale)
        if grad_hook is not None:
            grad_hook()
        self.optimizer_step()
        return loss.detach()

    @staticmethod
    def chunk_bounds(B: int, C: int):
        return [(k * B) // C for k in range(C + 1)]

    @staticmethod
    def chunk_seed(seed: int, k: int) -> int:
        """Tree / dropout seed of micro-batch k of the step with seed ``seed``."""
        return seed * 1009 + k + 1

    def _seed_nodes(self, users, pos, neg):
        u32, p32, n32 = (torch.as_tensor(t).to(device=self.device, dtype=torch.int32)
                         .contiguous() for t in (users, pos, neg))
        seeds = torch.empty(3 * u32.numel(), dtype=torch.int32, device=u32.device)
        check(lib.mirec_pack_seed_nodes(u32.data_ptr(), p32.data_ptr(), n32.data_ptr(),
                                        u32.numel(), self.n_user, seeds.data_ptr(),
                                        _lib.stream_handle()), "pack_seed_nodes")
        return seeds

    def _stage_chunks(self, users, pos, neg, seed, grad_hook, loss_scale, tree_hook, C,
                      chunk_hook):
        """The batch's B triples as C_eff = min(C, B) micro-batches of B_k
        triples.  Micro-batch k's loss is mean_k softplus + decay·all_param /
        B_k · s; its backward is seeded with loss_scale · B_k / B and s =
        1 / C_eff, so the summed gradients are exactly the whole batch's
        (Σ_k B_k/B · mean_k = mean over B; Σ_k B_k/B · s / B_k = 1/B) for any
        B, divisible by C or not; the returned loss is the same weighted sum.
        C_eff depends only on B, which every data-parallel rank shares (equal
        batch sizes), so every rank runs the same number of chunk hooks
        (collectives)."""
        users, pos, neg = (torch.as_tensor(t).to(self.device) for t in (users, pos, neg))
        B = int(users.numel())
        if B == 0:
            raise ValueError("empty batch")
        C = min(int(C), B)
        bnd = self.chunk_bounds(B, C)

        def sample(k):
            a, b = bnd[k], bnd[k + 1]
            return self.sample_tree(self._seed_nodes(users[a:b], pos[a:b], neg[a:b]),
                                    self.chunk_seed(seed, k))
        # sampled on first access, in order: the hook acts on tree k (issues
        # its row fetch) before tree k + 1 is sampled, so the fetch overlaps
        # the later trees' sampling and planning (each tree has its own seed:
        # the same trees as sampling them all first)
        trees = _ChunkTrees(sample, C)
        if tree_hook is not None:
            tree_hook(trees)
        one = self.__dict__.get("_loss_seed")
        if one is None or one.device != self.device:
            one = self._loss_seed = torch.ones((), dtype=torch.float32, device=self.device)
        total = torch.zeros((), device=self.device)
        for k, tree in enumerate(trees):
            chunk_hook(k, "pre")
            sk = self.chunk_seed(seed, k)
            w = (bnd[k + 1] - bnd[k]) / B
            emb = self.forward(tree, dropout_seed=sk if self.training else None)
            loss = self.loss_fused(emb, decay_scale=1.0 / C)
            with _BWD_ON_CALLER():
                loss.backward(one * (loss_scale * w))
            total += loss.detach() * w
            chunk_hook(k, "post")
        if grad_hook is not None:
            grad_hook()
        self.optimizer_step()
        return total

    def OneEpoch(self, user, pos, neg):
        B = int(self.config["bpr_batch_size"])
        n = len(user)
        user, pos, neg = (torch.as_tensor(t).to(self.device) for t in (user, pos, neg))
        acc = torch.zeros((), device=self.device)
        for i in range(0, n, B):
            acc += self.stageOne(user[i:i + B], pos[i:i + B], neg[i:i + B])
        return acc / (n // B + 1)

    def sample(self, n_triples: int, seed: int, offset: int = 0, shard: int = 0,
               n_shards: int = 1):
        u = torch.empty(n_triples, dtype=torch.int32, device=self.device)
        p, n = torch.empty_like(u), torch.empty_like(u)
        err = torch.zeros(1, dtype=torch.int32, device=self.device)
        sample_triples(self.graph, n_triples, seed, offset, u, p, n, err, shard, n_shards)
        self._sample_err = err
        return u, p, n

    # ----------------------------------------------------------- inference
    @torch.no_grad()
    def propagated(self) -> torch.Tensor:
        """Full-graph inference (getUsersRating 'all', graphsage.py:401-424):
        every node aggregates the mean of ALL its neighbours per layer."""
        self._check_table_current("propagated() / evaluation")
        x = self._table.detach()
        for i in range(self.num_layers):
            agg = torch.empty_like(x)
            csr_mean(self.graph, self._mean_dinv, x.contiguous(), agg)
            x = self.w_linears[i](torch.cat([x, agg], dim=1))
            if i != self.num_layers - 1:
                x = x.relu()
        return x

    @torch.no_grad()
    def eval_ratings(self):
        out = self.propagated()
        items = out[self.n_user:]
        return lambda users: out[users.long()] @ items.t()

    @torch.no_grad()
    def getUsersRating(self, users):
        return self.eval_ratings()(torch.as_tensor(users, device=self.device))
