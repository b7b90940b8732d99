"""Host-side logic on CPU: datasets / Loader parsing, metrics, the bench's
byte accounting, and the data-parallel driver over gloo (world_size 2) with
an oracle-backed engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import lightgcn_oracle as O


def test_loader_parses_reference_format(tmp_path):
    from furusato_recommend_amd import Loader
    d = tmp_path / "x"
    d.mkdir()
    (d / "trainx.txt").write_text("0 3 1 3\n1 2\n2 0 4\n")
    (d / "testx.txt").write_text("0 2\n2 1\n")
    ds = Loader({"suffix": "x"}, path=str(tmp_path))
    assert ds.n_users == 3 and ds.m_items == 5
    assert ds.trainUser.tolist() == [0, 0, 0, 1, 2, 2]
    assert ds.trainItem.tolist() == [3, 1, 3, 2, 0, 4]
    assert [a.tolist() for a in ds.allPos] == [[3, 1, 3], [2], [0, 4]]
    assert ds.testDict == {0: [2], 2: [1]}
    assert ds.trainDataSize == 6


def _write_random_file(path, rng, n_lines, max_items, messy):
    rows = []
    for k in range(n_lines):
        uid = k if not messy else int(rng.integers(0, n_lines * 2))
        items = rng.integers(0, 5000, int(rng.integers(1, max_items))).tolist()
        sep = "  " if (messy and k % 7 == 3) else " "
        tail = " " if (messy and k % 5 == 1) else ""
        rows.append(str(uid) + sep + sep.join(map(str, items)) + tail)
        if messy and k % 11 == 4:
            rows.append("")
    path.write_text("\n".join(rows) + ("\n" if messy else ""))


@pytest.mark.parametrize("n_lines,messy,test_mode", [(50, True, False), (300, True, True),
                                                     (60_000, False, False),
                                                     (60_000, True, True)])
def test_native_ingest_matches_reference_loop(tmp_path, n_lines, messy, test_mode):
    """mirec_parse_interactions (multi-threaded above 1 MiB) == the
    reference's line loop (oracle.parse_interaction_file), incl. repeated
    and trailing spaces, blank lines, no final newline, the test-mode cut."""
    from furusato_recommend_amd.dataloader import parse_interactions
    rng = np.random.default_rng(n_lines)
    f = tmp_path / "train.txt"
    _write_random_file(f, rng, n_lines, 40, messy)
    ref = O.parse_interaction_file(str(f), test_mode)
    uid, off, items, mu, mi = parse_interactions(str(f), 100 if test_mode else -1, n_threads=8)
    assert uid.tolist() == [u for u, _ in ref]
    got = [items[a:b].tolist() for a, b in zip(off[:-1], off[1:])]
    assert got == [it for _, it in ref]
    assert mu == max(u for u, _ in ref) and mi == max(max(it) for _, it in ref)


def test_native_ingest_rejects_malformed(tmp_path):
    from furusato_recommend_amd._lib import MirecError
    from furusato_recommend_amd.dataloader import parse_interactions
    f = tmp_path / "bad.txt"
    f.write_text("0 1 2\n1 3x 4\n")
    with pytest.raises(MirecError):
        parse_interactions(str(f))


def test_synthetic_invariants():
    from furusato_recommend_amd import FiveCore, SyntheticBipartite
    ds = SyntheticBipartite(1000, 200, 20000, seed=0)
    assert np.all(np.bincount(ds.trainUser, minlength=1000) >= 1)  # every uid has a line
    assert np.all(np.diff(ds.trainUser) >= 0)                       # grouped like the file
    assert len(ds.testDict) > 50
    for u, items in list(ds.testDict.items())[:50]:
        assert len(items) == 1
    z = SyntheticBipartite(1000, 200, 20000, seed=0, kind="zipf")
    cnt = np.bincount(z.trainItem, minlength=200)
    assert cnt[0] > 10 * np.median(cnt)
    fc = FiveCore(100, 50, 5)
    assert fc.trainDataSize == 400
    assert all(len(set(a.tolist())) == 4 for a in fc.allPos)


def test_metrics_match_oracle(golden):
    from furusato_recommend_amd import metric as M
    f = golden("metrics.npz")
    gt = [list(g) for g in np.split(f["gt_flat"], np.cumsum(f["gt_len"])[:-1])]
    r = M.getLabel(gt, f["pred"])
    assert np.array_equal(r, f["label"])
    res = M.test_one_batch(f["pred"], gt, (10, 20))
    assert np.allclose(res["recall"], [f["recall_at_10"], f["recall_at_20"]])
    assert np.allclose(res["ndcg"], [f["ndcg_at_10"], f["ndcg_at_20"]])
    assert np.allclose(res["precision"], [f["precision_at_10"], f["precision_at_20"]])


def test_algorithmic_bytes_c2():
    """10.69 GB per layer + the fused accumulate (acc read/write)."""
    from furusato_recommend_amd.engine import prop_launch_bytes
    N, nnz, D = 1_100_000, 40_000_000, 64
    mid = prop_launch_bytes(0, N, nnz, D, xs_out=True, addend=True, out=True)
    # neighbour rows 10.24 GB + col 0.16 + rowptr/dinv 0.013 + 3 x 0.2816 (acc r/w, x~ w)
    assert abs(mid / 1e9 - 11.258) < 1e-3
    survey = nnz * D * 4 + nnz * 4 + (N + 1) * 4 + N * 4 + N * D * 4
    assert abs(survey / 1e9 - 10.69) < 0.01
    fused_adam = prop_launch_bytes(0, N, nnz, D, slot=True, adam=True)
    assert fused_adam - prop_launch_bytes(0, N, nnz, D) == N * 4 + 6 * N * D * 4


# ------------------------------------------------------- data parallel (gloo)
class OracleEngine:
    """CPU stand-in with the PropagationEngine interface used by dist.py:
    dense mode via autograd; sparse mode via explicit seeds dL/d out (and
    the reg-gradient rows) + the linear backward sum_l Â^l d."""

    def __init__(self, o: O.OracleLightGCN, batch: int):
        self.o = o
        self.B3 = 3 * batch

    def forward(self, emb):
        return None

    def forward_for_batch(self, emb, users, pos, neg):
        return None

    def bpr(self, out, emb, users, pos, neg, decay, loss_accum=None, grad_scale=1.0):
        self._batch = (users, pos, neg)
        self._scale = grad_scale
        o = self.o
        N = o.emb.shape[0]
        e = o.emb.detach().clone().requires_grad_(True)
        out = O.forward(e, o.ei, o.n_users, o.L, o.div)
        out = torch.cat(out).detach().requires_grad_(True)
        u, p, n = (torch.as_tensor(x).long() for x in (users, pos, neg))
        us, ps, ns = out[u], out[p + o.n_users], out[n + o.n_users]
        loss = torch.mean(torch.nn.functional.softplus((us * ns).sum(1) - (us * ps).sum(1)))
        reg = 0.5 * (e[u].norm(2).pow(2) + e[p + o.n_users].norm(2).pow(2)
                     + e[n + o.n_users].norm(2).pow(2)) / float(len(u))
        (loss + decay * reg).backward()
        self._d = out.grad * grad_scale / (o.L + 1)
        self._e = e.grad * grad_scale
        self._N = N
        return (loss + decay * reg).detach()  # what the HIP bpr reports (stageOne's loss)

    def export_seeds(self):
        rows = torch.nonzero((self._d != 0).any(1) | (self._e != 0).any(1)).flatten()
        assert len(rows) <= self.B3
        keys = torch.full((self.B3,), self._N, dtype=torch.int32)
        rp = torch.zeros(self.B3, self._d.shape[1])
        re = torch.zeros_like(rp)
        keys[:len(rows)] = rows.int()
        rp[:len(rows)] = self._d[rows]
        re[:len(rows)] = self._e[rows]
        return keys, rp, re

    def import_seeds(self, keys, rows_p, rows_e):
        d = torch.zeros(self._N, rows_p.shape[1])
        e = torch.zeros_like(d)
        ok = keys < self._N
        d.index_add_(0, keys[ok].long(), rows_p[ok])
        e.index_add_(0, keys[ok].long(), rows_e[ok])
        self._d, self._e = d, e

    def static_row_lists(self, bm):
        return {"rows": bm.view(torch.uint8)[: self.o.emb.shape[0]].bool()}

    def invalidate_prescaled(self):
        pass

    def backward(self, emb, adam=None, grad_out=None, last_rows=None, on_chunk=None):
        if grad_out is not None:
            grad_out.copy_(self.o.grad(*self._batch) * self._scale)
            return
        g, x = self._d.clone(), self._d
        for _ in range(self.o.L):
            x = O.lgconv(x, self.o.ei, self.o.div)
            g = g + x
        before = self.o.emb.detach().clone()
        self.adam_step(emb, g + self._e, adam)
        if last_rows is not None:  # only this rank's shard is updated here
            chunks = last_rows if isinstance(last_rows, list) else [last_rows]
            keep = ~torch.stack([c["rows"] for c in chunks]).any(0)
            with torch.no_grad():
                self.o.emb[keep] = before[keep]
            for c in range(len(chunks)):
                if on_chunk is not None:
                    on_chunk(c)

    def adam_step(self, param, grad, adam):
        self.o.emb.grad = grad.clone()
        self.o.optim.step()
        self.o.emb.grad = None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dp_worker(rank, world, port, fpath, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import DataParallel
    f = dict(np.load(fpath))
    o = O.OracleLightGCN(f["train_user"], f["train_item"], int(f["n_users"]), int(f["m_items"]),
                         64, 3, float(f["lr"]), float(f["decay"]),
                         emb=torch.from_numpy(f["emb0"]) + (0.5 if rank else 0.0))
    t = f["triples"]
    half = len(t) // world
    # the broadcast in DataParallel fixes rank 1's perturbed init
    dp = DataParallel(OracleEngine(o, half), o.emb.data, None, mode=mode)
    for step in range(2):
        mine = t[rank * half:(rank + 1) * half]
        dp.step(mine[:, 0], mine[:, 1], mine[:, 2], float(f["decay"]))
    q.put((rank, o.emb.detach().numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sparse", "dense", "sharded"])
def test_data_parallel_equals_union_batch(golden, mode):
    """2 ranks on disjoint halves == one process on the union batch (the
    reference's own stageOne on all 64 triples = emb_step1/2), for both the
    sparse-seed all-gather and the dense-gradient all-reduce exchange."""
    from tests.conftest import GOLDEN
    fpath = os.path.join(GOLDEN, "lgcn_d64_L3.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, fpath, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    f = golden("lgcn_d64_L3.npz")
    assert np.array_equal(res[0], res[1])  # replicas stay identical
    ref = f["emb_step2"]
    assert np.max(np.abs(res[0] - ref)) / np.max(np.abs(ref)) < 2e-5


class _AccumEngine(OracleEngine):
    """OracleEngine that also sums the loss into the step's accumulator (as
    the HIP engine's bpr does)."""

    def bpr(self, out, emb, users, pos, neg, decay, loss_accum=None, grad_scale=1.0):
        loss = super().bpr(out, emb, users, pos, neg, decay, None, grad_scale)
        if loss_accum is not None:
            loss_accum += loss
        return loss


class _CpuLGCN(torch.nn.Module):
    """The model surface DPTrainer uses (state_dict, optim) over the oracle."""

    def __init__(self, o):
        super().__init__()
        self.o = o
        self.emb = o.emb
        self.optim = o.optim


def _dp_sampler(ds_pos, n_users, m_items, rank, world):
    """Rank-local triples from the rank's user shard, a rank-dependent count
    (the capped sampler keeps a data-dependent number per rank)."""
    def sample(epoch):
        rng = np.random.default_rng(1000 * epoch + rank)
        n = 40 + 7 * rank
        us = rng.integers(0, (n_users - rank + world - 1) // world, n) * world + rank
        u, p, ng = [], [], []
        for x in us:
            if len(ds_pos[x]) == 0:
                continue
            u.append(x)
            p.append(sorted(ds_pos[x])[rng.integers(0, len(ds_pos[x]))])
            while True:
                j = int(rng.integers(0, m_items))
                if j not in ds_pos[x]:
                    break
            ng.append(j)
        return np.array(u), np.array(p), np.array(ng)
    return sample


def _dp_trainer_worker(rank, world, port, fpath, ckpt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import DataParallel
    from furusato_recommend_amd.train_dp import DPTrainer
    f = dict(np.load(fpath))
    nu, mi = int(f["n_users"]), int(f["m_items"])
    tu, ti = f["train_user"], f["train_item"]
    pos = [set(ti[tu == k].tolist()) for k in range(nu)]
    test = {k: sorted(pos[k])[:1] for k in range(0, nu, 3) if pos[k]}

    class DS:
        n_users, m_items, trainDataSize, testDict = nu, mi, len(tu), test

    def make(seed_shift):
        o = O.OracleLightGCN(tu, ti, nu, mi, 64, 3, float(f["lr"]), float(f["decay"]),
                             emb=torch.from_numpy(f["emb0"]) + seed_shift)
        m = _CpuLGCN(o)
        dp = DataParallel(_AccumEngine(o, 16), o.emb.data, o.optim, mode="sparse")
        return o, m, dp

    def evaluator(model):
        with torch.no_grad():
            out = model.o.propagated()
        ue, ie = out[:nu], out[nu:]
        allpos = [np.array(sorted(s)) for s in pos]
        res = O.evaluate(ue, ie, test, allpos, topks=(10, 20))
        users = sorted(test)
        r = ue[torch.tensor(users)] @ ie.t()
        for i, u in enumerate(users):
            r[i, list(pos[u])] = -(1 << 10)
        return res, torch.topk(r, 20).indices.numpy()

    cfg = {"bpr_batch_size": 16, "decay": float(f["decay"]), "test_span": 1,
           "checkpoint_path": ckpt, "topks": (10, 20)}
    o, m, dp = make(0.5 if rank else 0.0)  # rank 1's init is overwritten by the broadcast
    sampler = _dp_sampler(pos, nu, mi, rank, world)
    seen = []

    def logged(ep):
        t = sampler(ep)
        seen.append(t)
        return t
    tr = DPTrainer(cfg, DS, m, dp=dp, sampler=logged, evaluator=evaluator)
    hist = tr.fit(2)
    final = o.emb.detach().numpy().copy()
    # resume: a fresh model (other init) from the checkpoint, then one more epoch
    o2, m2, dp2 = make(0.25)
    tr2 = DPTrainer(cfg, DS, m2, dp=dp2, sampler=sampler, evaluator=evaluator)
    loaded = tr2.load_checkpoint()
    resumed = (loaded, tr2.epoch, np.array_equal(o2.emb.detach().numpy(), final),
               all(torch.equal(a, b) for a, b in zip(
                   o2.optim.state[o2.emb].values(), o.optim.state[o.emb].values())))
    h2 = tr2.fit(1)
    q.put((rank, final, hist, seen, resumed, h2, o2.emb.detach().numpy().copy()))
    dist.destroy_process_group()


def test_dp_trainer_two_ranks_gloo(golden, tmp_path):
    """train_dp.DPTrainer (the ddp_lgcn.py:625-746 epoch driver) over the real
    DataParallel, 2 gloo ranks on CPU with the oracle-backed engine: two
    epochs with a barrier each, rank-local samples equalised to the same
    count, a checkpoint + evaluation (Recall / Precision / NDCG / HR /
    Coverage @10, @20) every epoch; replicas identical and equal to ONE
    oracle process stepping the union batches; the checkpoint reloads into
    a fresh model (table, Adam state, next epoch) and training resumes."""
    from tests.conftest import GOLDEN
    fpath = os.path.join(GOLDEN, "lgcn_d64_L3.npz")
    ckpt = str(tmp_path / "ckpt" / "ddp_lgn_all.pth")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_trainer_worker, args=(r, 2, port, fpath, ckpt, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=240)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    f = golden("lgcn_d64_L3.npz")
    (fin0, hist0, seen0, resumed0, h20, e20), (fin1, hist1, seen1, resumed1, h21, e21) = \
        res[0], res[1]
    assert np.array_equal(fin0, fin1) and np.array_equal(e20, e21)
    assert [h["epoch"] for h in hist0] == [0, 1] and [h["epoch"] for h in h20] == [2]
    for h in hist0:
        assert h["triples_per_rank"] == min(len(seen0[h["epoch"]][0]), len(seen1[h["epoch"]][0]))
        met = h["metrics"]
        for k in ("recall", "precision", "ndcg", "hr", "coverage"):
            assert len(met[k]) == 2 and all(np.isfinite(met[k]))
        assert 0 < met["coverage"][0] <= met["coverage"][1] <= 1
    assert hist1[0]["metrics"] is None  # rank 1 waits while rank 0 evaluates
    assert resumed0 == (True, 2, True, True) and resumed1 == (True, 2, True, True)
    assert hist0[0]["loss"] == hist1[0]["loss"]  # the union mean on every rank
    # one process stepping the union batches (rank-major) == the replicas
    nu, mi = int(f["n_users"]), int(f["m_items"])
    o = O.OracleLightGCN(f["train_user"], f["train_item"], nu, mi, 64, 3, float(f["lr"]),
                         float(f["decay"]), emb=torch.from_numpy(f["emb0"]))
    for ep in range(2):
        k = hist0[ep]["triples_per_rank"]
        for i in range(0, k, 16):
            j = min(i + 16, k)
            tri = [np.concatenate([seen0[ep][c][i:j], seen1[ep][c][i:j]]) for c in range(3)]
            o.stageOne(*tri)
    ref = o.emb.detach().numpy()
    assert np.max(np.abs(fin0 - ref)) / np.max(np.abs(ref)) < 2e-5
    assert os.path.exists(ckpt) and os.path.exists(ckpt + ".train")


def _write_split(golden, root):
    """The lgcn_d64_L3 fixture's graph as the reference's text files
    (dataloader.py:73-173: ``uid i1 i2 ...`` per line, suffix 'all')."""
    f = golden("lgcn_d64_L3.npz")
    tu, ti, nu = f["train_user"], f["train_item"], int(f["n_users"])
    d = root / "all"
    d.mkdir(parents=True)
    with open(d / "trainall.txt", "w") as fh:
        for u in range(nu):
            fh.write(" ".join(str(x) for x in [u, *ti[tu == u].tolist()]) + "\n")
    with open(d / "testall.txt", "w") as fh:
        for u in range(0, nu, 3):
            its = ti[tu == u]
            if len(its):
                fh.write(f"{u} {int(its[0])}\n")


def test_train_dp_cli_two_ranks_gloo(golden, tmp_path):
    """``python -m furusato_recommend_amd.train_dp --gpus 2`` (the mp.spawn
    entry point of ddp_lgcn.py:760-768): the parent starts
    torch.distributed.run as a child, the 2 ranks meet over gloo on CPU and
    run DPTrainer over the real DataParallel (the model plugin is the
    oracle-backed test model): an epoch, an evaluation, a checkpoint at
    <path>/ddp_lgn_all.pth; a second invocation resumes from it."""
    import json
    import subprocess
    import sys
    from tests.conftest import ROOT
    _write_split(golden, tmp_path / "data")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    ck = tmp_path / "ck"
    cmd = [sys.executable, "-m", "furusato_recommend_amd.train_dp", "--model", "lgn",
           "--gpus", "2", "--device", "cpu", "--data", str(tmp_path / "data"),
           "--recdim", "16", "--layer", "3", "--bpr_batch", "16", "--test_span", "1",
           "--path", str(ck), "--factory", "tests.dp_cli_factory:make", "--epochs"]
    runs = []
    for epochs in ("1", "1"):
        r = subprocess.run(cmd + [epochs], env=env, cwd=ROOT, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        runs.append([json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")])
    (a,), (b,) = runs  # rank 0 prints one line per epoch
    assert a["epoch"] == 0 and b["epoch"] == 1 and a["world"] == 2
    assert a["triples_per_rank"] > 0 and np.isfinite(a["loss"])
    for rec in (a, b):
        for k in ("recall", "precision", "ndcg", "hr", "coverage"):
            assert len(rec["metrics"][k]) == 2 and all(np.isfinite(rec["metrics"][k]))
    p = ck / "ddp_lgn_all.pth"
    assert p.exists()
    assert torch.load(str(p) + ".train", weights_only=True)["epoch"] == 1


def test_pos_cdf_build_matches_numpy_choice(golden):
    """mirec_pos_cdf_build (host, libmirec) == numpy choice's normalised
    cumulative probabilities per user row (oracle.pos_cdf), in float64 —
    exactly, each row ending at exactly 1; bad rows rejected; a long tail of
    tiny probabilities keeps one CDF step per entry (a float CDF
    merged entries below ~2^-24 of the row mass into their neighbours)."""
    import ctypes

    from furusato_recommend_amd import Graph
    from furusato_recommend_amd._lib import lib
    f = golden("sampler_weighted.npz")
    u, i, nu, mi = f["train_user"], f["train_item"], int(f["n_users"]), int(f["m_items"])
    all_pos = [i[u == k] for k in range(nu)]
    flat = np.ascontiguousarray(f["probs_flat"], np.float64)
    probs = np.split(flat, np.cumsum([len(p) for p in all_pos])[:-1])
    g = Graph.from_interactions(u, i, nu, mi, "cpu")
    rp = g.rowptr_host
    # the CSR's user rows are the allPos order
    assert all(np.array_equal(g.col_host[rp[k]:rp[k + 1]] - nu, all_pos[k]) for k in range(nu))
    cdf = np.empty(len(flat), np.float64)
    assert lib.mirec_pos_cdf_build(rp.ctypes.data, nu, flat.ctypes.data, cdf.ctypes.data) == 0
    ref = O.pos_cdf(all_pos, probs)
    assert np.array_equal(cdf, ref)
    ends = rp[1:nu + 1] - rp[0] - 1
    assert np.all(cdf[ends[np.diff(rp[:nu + 1]) > 0]] == 1.0)
    for k in range(nu):
        seg = cdf[rp[k] - rp[0]:rp[k + 1] - rp[0]]
        assert np.all(np.diff(seg) >= 0)
    bad = flat.copy()
    bad[0] = -0.1
    assert lib.mirec_pos_cdf_build(rp.ctypes.data, nu, bad.ctypes.data, cdf.ctypes.data) != 0
    bad = flat.copy()
    bad[rp[0]:rp[1]] = 0.0  # a row of zeros
    assert lib.mirec_pos_cdf_build(rp.ctypes.data, nu, bad.ctypes.data, cdf.ctypes.data) != 0
    # the Python entry point: per-user arrays, sizes checked
    g.set_positive_probs(probs)
    assert np.array_equal(g.pos_cdf.numpy(), cdf)
    with pytest.raises(ValueError):
        g.set_positive_probs(probs[:-1])
    # the long tail: 1e-12 entries between two halves stay distinct steps
    tail = np.array([0.5] + [1e-12] * 6 + [0.5])
    trp = np.array([0, len(tail)], dtype=np.int64)
    tc = np.empty(len(tail), np.float64)
    assert lib.mirec_pos_cdf_build(trp.ctypes.data, 1, tail.ctypes.data, tc.ctypes.data) == 0
    assert np.all(np.diff(tc) > 0) and tc[-1] == 1.0
    assert np.array_equal(tc, np.cumsum(tail) / np.cumsum(tail)[-1])
    assert np.any(np.diff(tc.astype(np.float32)) == 0)  # what a float CDF would have merged
    _ = ctypes


def test_train_dp_cli_launch_command():
    """The launcher's child command and environment (no processes)."""
    from furusato_recommend_amd import train_dp as T
    a = T.parse_args(["--model", "sage", "--gpus", "8"])
    assert T.needs_launch(a, env={}) and not T.needs_launch(a, env={"WORLD_SIZE": "8"})
    assert not T.needs_launch(T.parse_args([]), env={})
    seen = {}

    class R:
        returncode = 3
    assert T.launch(a, ["--model", "sage", "--gpus", "8"],
                    runner=lambda cmd, env: seen.update(cmd=cmd, env=env) or R()) == 3
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("-m", 3):][:2] == ["-m", "furusato_recommend_amd.train_dp"]
    assert cmd[-4:] == ["--model", "sage", "--gpus", "8"]
    # the rendezvous store binds its own port: no port picked and handed over
    assert "--rdzv-endpoint=127.0.0.1:0" in cmd and "--local-addr=127.0.0.1" in cmd
    assert "--master-port" not in cmd
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    cfg = T.build_config(T.parse_args(["--model", "sage", "--suffix", "x", "--path", "/c"]), "cuda:0")
    assert cfg["checkpoint_path"] == "/c/ddp_sage_x.pth" and cfg["topks"] == (10, 20)
    assert cfg["bpr_batch_size"] == 20000 and cfg["decay"] == 1e-4 and cfg["lr"] == 1e-3


def _calib_worker(rank, world, port, fpath, q, prefer):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import DataParallel
    f = dict(np.load(fpath))
    o = O.OracleLightGCN(f["train_user"], f["train_item"], int(f["n_users"]), int(f["m_items"]),
                         64, 3, float(f["lr"]), float(f["decay"]), emb=torch.from_numpy(f["emb0"]))
    t = f["triples"]
    half = len(t) // world
    mine = t[rank * half:(rank + 1) * half]
    dp = DataParallel(OracleEngine(o, half), o.emb.data, o.optim, mode="auto", chunks=3)
    assert dp.mode == "sparse"  # until measured
    dp.adam = _OptimView(o)
    seen = []

    def run_step():
        seen.append(dp.mode)
        dp.step(mine[:, 0], mine[:, 1], mine[:, 2], float(f["decay"]))

    def measure(mode, fn, steps):  # rank-dependent fake clock: max over ranks decides
        for _ in range(steps):
            fn()
        fast = 1.0 if mode == prefer else 2.0
        return dp._max_over_ranks(fast + 0.5 * rank)
    cal = dp.calibrate(run_step, steps=1, measure=measure)
    stale_after = dp.adam.stale_rows
    run_step()
    q.put((rank, o.emb.detach().numpy().copy(), cal, seen, stale_after,
           dp.adam.exp_avg.numpy().copy()))
    dist.destroy_process_group()


class _OptimView:
    """The oracle's torch.optim.Adam seen as an AdamState (moments by view)."""

    def __init__(self, o):
        self.o = o
        self.stale_rows = False
        o.emb.grad = torch.zeros_like(o.emb)
        o.optim.step()  # materialise the state tensors (a zero step leaves emb unchanged) ...
        o.emb.grad = None
        st = o.optim.state[o.emb]
        st["step"].zero_()  # ... and forget it happened
        st["exp_avg"].zero_()
        st["exp_avg_sq"].zero_()
        self.exp_avg, self.exp_avg_sq = st["exp_avg"], st["exp_avg_sq"]


@pytest.mark.parametrize("prefer", ["sparse", "sharded"])
def test_data_parallel_auto_calibration(golden, prefer):
    """mode="auto": both exchanges are timed on the ranks (max over ranks),
    the faster one is kept, and every calibration step is an ordinary
    training step: after 2 + 2 calibration steps and one more, both ranks
    hold 5 union-batch steps of the reference (and, leaving ``sharded``, the
    gathered Adam moments)."""
    from tests.conftest import GOLDEN
    fpath = os.path.join(GOLDEN, "lgcn_d64_L3.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_worker, args=(r, 2, port, fpath, q, prefer))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=180) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    f = golden("lgcn_d64_L3.npz")
    o = O.OracleLightGCN(f["train_user"], f["train_item"], int(f["n_users"]), int(f["m_items"]),
                         64, 3, float(f["lr"]), float(f["decay"]), emb=torch.from_numpy(f["emb0"]))
    t = f["triples"]
    for _ in range(5):
        o.stageOne(t[:, 0], t[:, 1], t[:, 2])
    ref = o.emb.detach().numpy()
    for r in (0, 1):
        emb, cal, seen, stale, mom = res[r]
        assert cal["choice"] == prefer
        assert cal["sparse_ms_per_step"] == (1.5 if prefer == "sparse" else 2.5)
        assert seen == ["sparse", "sparse", "sharded", "sharded", prefer]
        assert not stale
        assert np.max(np.abs(emb - ref)) / np.max(np.abs(ref)) < 2e-5
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][4], res[1][4])  # moments agree on every row


def _dense_dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import DenseGradDataParallel

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            g = torch.Generator().manual_seed(rank)  # replicas start different
            self.table = torch.nn.Parameter(torch.randn(1 << 20 | 8, 4, generator=g))
            self.lin = torch.nn.Linear(4, 3)

    m = M()
    dp = DenseGradDataParallel(m)
    for k, p in enumerate(m.parameters()):
        p.grad = torch.full_like(p, float(rank + 1) * (k + 1))
    dp._allreduce()
    # numpy, not tensors: torch shares tensor storage through a file
    # descriptor that dies with this process
    q.put((rank, [p.detach().numpy().copy() for p in m.parameters()],
           [p.grad.numpy().copy() for p in m.parameters()]))
    dist.destroy_process_group()


def test_dense_grad_data_parallel_gloo():
    """DenseGradDataParallel (GraphSAGE / SASRec DP): rank-0 broadcast of the
    parameters, SUM all-reduce of every gradient (the big table in place, the
    small ones through the flattened bucket)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (ps, gs) for r, ps, gs in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    for a, b in zip(res[0][0], res[1][0]):
        assert np.array_equal(a, b)
    for k, (a, b) in enumerate(zip(res[0][1], res[1][1])):
        assert np.array_equal(a, b) and np.all(a == 3.0 * (k + 1))


def test_split_k_linear_matches_nn_linear():
    """linear.Linear (split-K weight gradient, used on packed activations) ==
    nn.Linear in value and in every gradient, above and below the split
    threshold and with a ragged tail."""
    from furusato_recommend_amd.linear import Linear, weight_grad
    torch.manual_seed(0)
    for n in (100, 8192, 20_011):
        x = torch.randn(n, 128, dtype=torch.float64, requires_grad=True)
        a = Linear(128, 96).double()
        b = torch.nn.Linear(128, 96).double()
        b.load_state_dict(a.state_dict())
        x2 = x.detach().clone().requires_grad_(True)
        gy = torch.randn(n, 96, dtype=torch.float64)
        ya, yb = a(x), b(x2)
        assert torch.allclose(ya, yb)
        ya.backward(gy)
        yb.backward(gy)
        assert torch.allclose(x.grad, x2.grad)
        assert torch.allclose(a.weight.grad, b.weight.grad, rtol=1e-10, atol=1e-9)
        assert torch.allclose(a.bias.grad, b.bias.grad)
        assert torch.allclose(weight_grad(gy, x.detach()), gy.t() @ x.detach())


def test_length_buckets_order_and_counts():
    """Host bucketing of the packed SASRec batch: stable order by
    ceil(len/16) clipped to 1..4 (length 0 joins bucket 1), counts that
    partition the batch, and every sequence inside its bucket's row limit."""
    from furusato_recommend_amd.sasrec import length_buckets
    rng = np.random.default_rng(0)
    for lens in ([0, 1, 16, 17, 32, 33, 48, 49, 64], rng.integers(0, 65, 1000), [50] * 5, [3]):
        lens = np.asarray(lens)
        order, be = length_buckets(lens)
        assert sorted(order.tolist()) == list(range(len(lens)))
        assert len(be) == 4 and be[3] == len(lens) and list(be) == sorted(be)
        lo = 0
        for k, hi in enumerate(be):
            seg = order[lo:hi]
            assert (lens[seg] <= 16 * (k + 1)).all()
            assert (np.diff(seg) > 0).all()  # stable inside a bucket
            lo = hi


def test_bench_launcher_command():
    """`python bench.py --gpus N` with no WORLD_SIZE starts N ranks itself
    (torch.distributed.run as a child; ddp_lgcn.py:760-768 mp.spawn) and
    returns their exit status; under a launcher it runs as a rank."""
    import bench
    a = bench.parse(["--gpus", "4", "--steps", "3"])
    assert bench.needs_launch(a, env={})
    assert not bench.needs_launch(a, env={"WORLD_SIZE": "4"})
    assert not bench.needs_launch(bench.parse([]), env={})
    seen = {}

    class R:
        returncode = 7

    def runner(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return R()
    assert bench.launch(a, ["--gpus", "4", "--steps", "3"], runner=runner) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--rdzv-endpoint=127.0.0.1:0" in cmd
    assert "--local-addr=127.0.0.1" in cmd and "--master-port" not in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:] and cmd[-4] == "--gpus"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_self_launch_two_ranks_gloo():
    """The real process tree on CPU: the parent spawns 2 ranks, they meet
    over gloo (with the watchdog timeout), rank 0 prints one JSON line."""
    import json
    import subprocess
    import sys
    from tests.conftest import ROOT
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--launch-selftest"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    assert json.loads(lines[0]) == {"n_gpus": 2, "sum": 3.0}


def test_bench_oracle_parity_leg():
    """bench.py's parity leg: the oracle takes the snapshot's step from the
    snapshot's table, Adam moments and step count.  A snapshot whose "GPU"
    half is another oracle taking the same step from the same state passes
    with zero error; a perturbed table or loss fails the 1e-4 bar."""
    import bench
    from oracle.lightgcn_oracle import OracleLightGCN
    rng = np.random.default_rng(3)
    nu, mi, E, D = 60, 40, 500, 16
    tu, ti = rng.integers(0, nu, E), rng.integers(0, mi, E)
    trip = (rng.integers(0, nu, 32), rng.integers(0, mi, 32), rng.integers(0, mi, 32))
    a = OracleLightGCN(tu, ti, nu, mi, D, 3, 1e-3, 1e-4, seed=1)
    for _ in range(3):  # non-trivial Adam state
        a.stageOne(*trip)
    st = a.optim.state[a.emb]
    snap = {"emb0": a.emb.detach().clone(), "exp_avg": st["exp_avg"].clone(),
            "exp_avg_sq": st["exp_avg_sq"].clone(), "n_steps": int(st["step"]),
            "lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8, "out_gpu": a.propagated(),
            "users": trip[0], "pos": trip[1], "neg": trip[2], "step_index": 3}
    snap["loss_gpu"] = a.stageOne(*trip)
    snap["emb1_gpu"] = a.emb.detach().clone()
    fresh = OracleLightGCN(tu, ti, nu, mi, D, 3, 1e-3, 1e-4, seed=9)  # other init: overwritten
    r = bench.oracle_parity(fresh, snap)
    assert r["ok"] and r["rel_out"] == 0.0 and r["rel_emb_step"] == 0.0 and r["rel_loss"] == 0.0
    snap["emb1_gpu"] = snap["emb1_gpu"] + 1e-3 * snap["emb1_gpu"].abs().max()
    r = bench.oracle_parity(OracleLightGCN(tu, ti, nu, mi, D, 3, 1e-3, 1e-4), snap)
    assert not r["ok"] and r["rel_emb_step"] > 1e-4 and r["rel_out"] == 0.0


class _StepView(_OptimView):
    """_OptimView with the AdamState fields the parity leg snapshots."""

    def __init__(self, o, lr):
        super().__init__(o)
        self.lr, self.betas, self.eps = lr, (0.9, 0.999), 1e-8

    @property
    def n_steps(self):
        return int(self.o.optim.state[self.o.emb]["step"])


def _bench_dp_legs_worker(rank, world, port, fpath, q, mode, tamper):
    """One rank of bench.py's N > 1 legs over gloo with the oracle engine:
    two ordinary data-parallel steps, the parity leg (dp_union_parity, rank 0
    replaying the union batch on a fresh oracle), then the quality loop
    (train_then_evaluate: every rank steps, rank 0 evaluates)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from furusato_recommend_amd.dist import DataParallel
    f = dict(np.load(fpath))
    nu, mi, lr, decay = int(f["n_users"]), int(f["m_items"]), float(f["lr"]), float(f["decay"])
    o = O.OracleLightGCN(f["train_user"], f["train_item"], nu, mi, 64, 3, lr, decay,
                         emb=torch.from_numpy(f["emb0"]))
    t = f["triples"]
    per = len(t) // world
    dp = DataParallel(OracleEngine(o, per), o.emb.data, None, mode=mode, chunks=2)
    view = _StepView(o, lr)
    dp.adam = view

    def batch(i):
        b = np.roll(t, 7 * i, axis=0)[rank * per:(rank + 1) * per]
        return b[:, 0], b[:, 1], b[:, 2]
    for i in range(2):
        dp.step(*batch(i), decay)
    if tamper == "replica" and rank == 1:
        with torch.no_grad():
            o.emb[3, 5] += 1e-3  # this replica drifts: the digests must disagree

    def replay(snap, U, P, N):
        r = O.OracleLightGCN(f["train_user"], f["train_item"], nu, mi, 64, 3, lr, decay,
                             emb=snap["emb0"])
        r.optim.state[r.emb] = {"step": torch.tensor(float(snap["n_steps"])),
                                "exp_avg": snap["exp_avg"].clone(),
                                "exp_avg_sq": snap["exp_avg_sq"].clone()}
        loss = r.stageOne(U.numpy(), P.numpy(), N.numpy())
        e = r.emb.detach()
        if tamper == "replay":
            e = e + 1e-3 * e.abs().max()
        return e, loss
    par = bench.dp_union_parity(dp, o.emb.data, view, *batch(2), decay, replay)
    seen = []

    def step(i):
        seen.append(i)
        dp.step(*batch(3 + i), decay)
    ev, _ = bench.train_then_evaluate(step, 3, lambda: {"emb": o.emb.detach().numpy().copy()},
                                      rank, world)
    q.put((rank, par, ev, seen, o.emb.detach().numpy().copy()))
    dist.destroy_process_group()


def _run_dp_legs(mode, tamper=None, world=2):
    from tests.conftest import GOLDEN
    fpath = os.path.join(GOLDEN, "lgcn_d64_L3.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_dp_legs_worker,
                         args=(r, world, port, fpath, q, mode, tamper)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("mode", ["sparse", "sharded"])
def test_bench_dp_parity_and_quality_legs_gloo(mode):
    """bench.py at N > 1 proves itself: after ordinary
    data-parallel steps, one more step leaves bitwise-equal replicas (table
    and gathered Adam moments, compared by all-gathered digests) and rank 0's
    replay of ONE single-process step on the union batch from the snapshot
    matches the data-parallel table at 1e-4; the quality loop steps every rank
    and evaluates on rank 0 only."""
    res = _run_dp_legs(mode)
    par0, ev0, seen0, emb0 = res[0]
    par1, ev1, seen1, emb1 = res[1]
    assert par0["ok"], par0
    assert par0["replicas_bitwise_equal"] and par0["moments_bitwise_equal"]
    assert par0["rel_emb_step"] < 2e-5 and par0["rel_loss"] < 1e-5
    assert par0["union_batch"] == 64 and par0["mode"] == mode
    assert par1["table_digest"] == par0["table_digest"] and "ok" not in par1
    assert seen0 == seen1 == [0, 1, 2]
    assert ev1 is None and np.array_equal(ev0["emb"], emb0)
    assert np.array_equal(emb0, emb1)


@pytest.mark.parametrize("tamper", ["replica", "replay"])
def test_bench_dp_parity_leg_detects_divergence(tamper):
    """A drifted replica fails the bitwise digest check; a union replay that
    disagrees fails the 1e-4 bar."""
    par0 = _run_dp_legs("sparse", tamper)[0][0]
    assert not par0["ok"]
    if tamper == "replica":
        assert not par0["replicas_bitwise_equal"]
    else:
        assert par0["replicas_bitwise_equal"] and par0["rel_emb_step"] > 1e-4


def test_chunk_trees_negative_index():
    """_ChunkTrees[-1] is the last micro-batch tree (sampling the earlier
    ones first); out of range raises."""
    from furusato_recommend_amd.graphsage import _ChunkTrees
    seen = []
    t = _ChunkTrees(lambda j: seen.append(j) or f"t{j}", 3)
    assert t[-1] == "t2" and seen == [0, 1, 2]
    assert t[-3] == "t0" and list(t) == ["t0", "t1", "t2"]
    for k in (3, -4):
        with pytest.raises(IndexError):
            t[k]


def test_host_threads_bounded():
    import bench
    n = bench.host_threads()
    assert 1 <= n <= (os.cpu_count() or 1)


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import DataParallel

    class Eng:
        def static_row_lists(self, bm):
            return {"bm": bm}
    N, D = 11, 3
    emb = torch.zeros(N, D)
    dp = DataParallel(Eng(), emb, None, mode="sharded")
    t = torch.full((N, D), -1.0)
    t[rank:N:world] = torch.arange(N, dtype=torch.float32)[rank:N:world, None] * 10 + rank
    dp._gather_rows(t)
    q.put((rank, t.numpy().copy()))
    dist.destroy_process_group()


def test_sharded_gather_rows_ragged_world3():
    """The sharded mode's all-gather of interleaved row shards (row i owned by
    rank i mod W) at W = 3 with N = 11 rows (a ragged last block): every rank
    ends with every owner's rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    want = (np.arange(11) * 10 + np.arange(11) % 3).astype(np.float32)
    for r in range(3):
        assert np.array_equal(res[r][:, 0], want) and np.array_equal(res[r][:, 2], want)


def test_csr_sort_rows_matches_numpy():
    """mirec_csr_sort_rows (host, threaded): each user row sorted ascending,
    multi-edges kept — the samplers' binary-search rows."""
    from furusato_recommend_amd import _lib
    rng = np.random.default_rng(2)
    n_rows = 3000
    deg = rng.integers(0, 90, n_rows)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = rng.integers(0, 500, int(rowptr[-1])).astype(np.int32)
    out = np.empty_like(col)
    _lib.check(_lib.lib.mirec_csr_sort_rows(rowptr.ctypes.data, col.ctypes.data, n_rows,
                                            out.ctypes.data), "sort_rows")
    for r in range(n_rows):
        assert np.array_equal(out[rowptr[r]:rowptr[r + 1]], np.sort(col[rowptr[r]:rowptr[r + 1]]))


def test_host_code_under_asan_ubsan(tmp_path):
    """The host C++ of libmirec (graph build, row sort, long-row schedule,
    text ingest) built with AddressSanitizer + UBSan and run on random and
    malformed inputs (tests/native/host_check.cpp)."""
    import shutil
    import subprocess
    from tests.conftest import ROOT
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    src = os.path.join(ROOT, "furusato_recommend_amd", "csrc")
    exe = str(tmp_path / "host_check")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-pthread",
           "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "native", "host_check.cpp"),
           os.path.join(src, "graph.cpp"), os.path.join(src, "ingest.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "host_check ok" in r.stdout


def test_torch_ops_registration_and_fake_tracing():
    """torch.ops.mirec.lgcn_propagate / _t are registered operators with
    autograd and fake (meta) implementations: shape propagation under
    FakeTensorMode runs no kernel (SURVEY §8b operator API)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode

    import furusato_recommend_amd  # noqa: F401  (registers the ops)
    from furusato_recommend_amd import ops
    assert hasattr(torch.ops.mirec, "lgcn_propagate") and hasattr(torch.ops.mirec, "lgcn_propagate_t")

    class _G:
        n_nodes, symmetric = 7, True
    g = _G()
    h = ops.handle(g)
    assert ops.handle(g) == h
    with FakeTensorMode():
        x = torch.empty(7, 16)
        y = torch.ops.mirec.lgcn_propagate(x, h)
        yt = torch.ops.mirec.lgcn_propagate_t(x, h)
    assert y.shape == (7, 16) and yt.shape == (7, 16)
    import pytest
    with pytest.raises(ValueError):
        torch.ops.mirec.lgcn_propagate(torch.empty(7, 16), h)  # not on the HIP device


def _route_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from furusato_recommend_amd.dist import route_rows
    n_rows, d = 12, 3
    g = torch.Generator().manual_seed(rank)
    rows = torch.sort(torch.randperm(n_rows, generator=g)[: 4 + 2 * rank]).values.int()
    vals = rows.float()[:, None] * 10 + rank + torch.arange(d).float()[None] / 10
    rid, rv, counts = route_rows(rows, vals, n_rows)
    q.put((rank, rows.numpy(), rid.numpy(), rv.numpy(), counts))
    dist.destroy_process_group()


def test_route_rows_to_owners_world3():
    """route_rows (the routed table exchange of DenseGradDataParallel): at
    W = 3 over 12 rows every (row, value) reaches the owner of its
    contiguous block, in source-rank order, ascending within a source."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_route_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(3))}
    for p in procs:
        p.join(timeout=60)
    for owner in range(3):
        _, rid, rv, counts = res[owner]
        want_ids, want_vals = [], []
        for src in range(3):
            rows = res[src][0]
            mine = rows[(rows // 4) == owner]
            want_ids += mine.tolist()
            want_vals += [[r * 10 + src + k / 10 for k in range(3)] for r in mine]
            assert counts[src] == len(mine)
        assert rid.tolist() == want_ids
        assert np.allclose(rv, np.array(want_vals, dtype=np.float32).reshape(-1, 3))


def _bf16_rne(x: np.ndarray) -> np.ndarray:
    """f32 -> nearest bf16 (ties to even), returned as f32 — what
    v_cvt_pk_bf16_f32 does for finite values."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def test_bf16_three_term_split_error_bound():
    """The GEMMs' f32 products on bf16 MFMA (csrc/common.h split3, gemm.hip
    MIREC_GEMM_X6), emulated on the host: x = x_h + x_m + x_l with every
    residual exact in f32, |x_m| <= 2^-8 |x|, |x_l| <= 2^-16 |x|, the split
    exact to 2^-24 |x|, and the six kept products (a_l b_h + a_h b_l + a_m b_m
    + a_m b_h + a_h b_m + a_h b_h, exact in float64 as bf16 x bf16 products
    are) within 2^-22 |a b| of the exact product — an f32 rounding's order."""
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200_000) * 10.0 ** rng.uniform(-30, 30, 200_000)).astype(np.float32)
    y = (rng.standard_normal(200_000) * 10.0 ** rng.uniform(-30, 30, 200_000)).astype(np.float32)

    def split(v):
        h = _bf16_rne(v)
        r1 = (v - h).astype(np.float32)
        m = _bf16_rne(r1)
        r2 = (r1 - m).astype(np.float32)
        lo = _bf16_rne(r2)
        # the residuals are exact: recomputing in float64 gives the same
        assert np.array_equal(r1.astype(np.float64), v.astype(np.float64) - h.astype(np.float64))
        assert np.array_equal(r2.astype(np.float64), r1.astype(np.float64) - m.astype(np.float64))
        return h.astype(np.float64), m.astype(np.float64), lo.astype(np.float64)
    xh, xm, xl = split(x)
    yh, ym, yl = split(y)
    ax = np.abs(x.astype(np.float64))
    assert np.all(np.abs(xm) <= 2.0 ** -8 * ax) and np.all(np.abs(xl) <= 2.0 ** -16 * ax)
    assert np.all(np.abs(xh + xm + xl - x.astype(np.float64)) <= 2.0 ** -24 * ax)
    six = xl * yh + xh * yl + xm * ym + xm * yh + xh * ym + xh * yh
    exact = x.astype(np.float64) * y.astype(np.float64)
    rel = np.abs(six - exact) / np.abs(exact)
    assert rel.max() <= 2.0 ** -22, rel.max()


# ---------------------------------------------- configuration C1 on the host
class _DS:
    def __init__(self, u, i, nu, mi):
        self.trainUser, self.trainItem = np.asarray(u), np.asarray(i)
        self.n_users, self.m_items = int(nu), int(mi)
        self.trainDataSize = len(u)


def test_mf_cpu_step_matches_reference_fixture(golden):
    """C1's host path (mirec_cpu_bpr_step: model/MF.py:62-94 + torch Adam)
    against the reference MF's own step (mf_d32.npz, make_golden.py): the
    returned loss, both tables after the step, getUsersRating after it."""
    from furusato_recommend_amd import MF
    f = golden("mf_d32.npz")
    m = MF({"latent_dim_rec": 32, "lr": float(f["lr"]), "decay": float(f["decay"]),
            "device": "cpu", "bpr_batch_size": 64},
           _DS(f["train_user"], f["train_item"], f["n_users"], f["m_items"]))
    m.load_table(torch.from_numpy(f["user_w0"]), torch.from_numpy(f["item_w0"]))
    t = torch.from_numpy(f["triples"])
    loss, reg = m.bpr_loss(t[:, 0], t[:, 1], t[:, 2])
    assert abs(float(loss) - float(f["loss"])) < 1e-5 * abs(float(f["loss"]))
    sl = float(m.stageOne(t[:, 0], t[:, 1], t[:, 2]))
    assert abs(sl - float(f["step_loss"])) < 1e-5 * abs(float(f["step_loss"]))

    def rel(a, b):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        return float(np.abs(a - b).max() / np.abs(b).max())
    assert rel(m.embedding_user.weight.detach(), f["user_w1"]) < 1e-6
    assert rel(m.embedding_item.weight.detach(), f["item_w1"]) < 1e-6
    assert rel(m.getUsersRating(torch.arange(5)), f["rating5"]) < 1e-6


def test_mf_cpu_c1_epochs_and_evaluation_vs_oracle():
    """BASELINE C1 as stated (10 000 users x 1 000 items, 5-core, d = 32,
    CPU single-process): the model's own host sampler (triples the device
    sampler draws too) and two OneEpochs against OracleMF stepping the same
    triples (loss, tables at 1e-5), then evaluate() on the host == the
    oracle's Trainer.test arithmetic (trainer.py:115-170) on the same tables."""
    from furusato_recommend_amd import MF, FiveCore
    from furusato_recommend_amd.evaluate import evaluate
    ds = FiveCore(10_000, 1_000, 5, seed=0)
    torch.manual_seed(2020)
    m = MF({"latent_dim_rec": 32, "lr": 1e-3, "decay": 1e-4, "device": "cpu",
            "bpr_batch_size": 2048, "n_threads": 4}, ds)
    o = O.OracleMF(m.embedding_user.weight, m.embedding_item.weight, 1e-3, 1e-4)
    for ep in range(2):
        u, p, n = m.sample(ds.trainDataSize, seed=2020, offset=ep * ds.trainDataSize)
        assert int(m._sample_err) == 0
        uu, pp, nn_ = u.numpy(), p.numpy(), n.numpy()
        for k in range(0, len(uu), 331):  # the sampler's invariants
            assert pp[k] in ds.allPos[uu[k]] and nn_[k] not in ds.allPos[uu[k]]
        lg = float(m.OneEpoch(u, p, n))
        acc = 0.0
        for i in range(0, len(uu), 2048):
            acc += o.stageOne(uu[i:i + 2048], pp[i:i + 2048], nn_[i:i + 2048])
        lo = acc / (len(uu) // 2048 + 1)
        assert abs(lg - lo) < 1e-5 * abs(lo)
        for a, b in ((m.embedding_user.weight, o.user), (m.embedding_item.weight, o.item)):
            a, b = a.detach().double(), b.detach().double()
            assert float((a - b).abs().max() / b.abs().max()) < 1e-5
    # the host sampler is a pure function of (seed, offset): shape-independent
    u2, _, _ = m.sample(1000, seed=2020, offset=500)
    u1, _, _ = m.sample(2000, seed=2020, offset=0)
    assert torch.equal(u2, u1[500:1500])
    res, top = evaluate(m, ds.testDict, (10, 20), 4000, return_topk=True)
    allpos = [np.asarray(a) for a in ds.allPos]
    ref = O.evaluate(o.user.detach(), o.item.detach(), ds.testDict, allpos, topks=(10, 20))
    for k in ("recall", "precision", "ndcg"):
        assert np.allclose(res[k], ref[k], atol=2e-4), (k, res[k], ref[k])


def test_host_capped_sampler_matches_sequential_rule():
    """mirec_cpu_bpr_sample_capped (the ddp_lgcn.py epoch sampler for a CPU
    model) == the reference's loop (ddp_lgcn.py:541-582) on the
    same candidate stream: users without positives skipped, a candidate kept
    iff its positive was kept < cap times before it, kept triples in draw
    order, negatives never positives; sharded streams stay in the shard."""
    from furusato_recommend_amd import SyntheticBipartite
    from furusato_recommend_amd.engine import sample_epoch_capped
    from furusato_recommend_amd.graph import Graph
    ds = SyntheticBipartite(3000, 400, 30_000, seed=4, kind="zipf", test_frac=0)
    g = Graph.from_interactions(ds.trainUser, ds.trainItem, ds.n_users, ds.m_items, "cpu")
    cap = 40
    for shard, n_shards in ((0, 1), (1, 3)):
        u, p, n, cu, cp = sample_epoch_capped(g, 3 * 30_000, cap, seed=9, shard=shard,
                                              n_shards=n_shards, return_candidates=True,
                                              n_threads=4)
        assert u.device.type == "cpu"
        cu, cp = cu.numpy(), cp.numpy()
        cnt, kept = {}, []
        for t in range(len(cp)):
            if cp[t] < 0 or cnt.get(int(cp[t]), 0) >= cap:
                continue
            cnt[int(cp[t])] = cnt.get(int(cp[t]), 0) + 1
            kept.append(t)
        kept = np.array(kept)
        assert len(kept) == u.numel() and len(kept) < len(cp)  # the cap bit
        assert np.array_equal(u.numpy(), cu[kept]) and np.array_equal(p.numpy(), cp[kept])
        assert (u.numpy() % n_shards == shard).all()
        rp, col = g.rowptr_host, g.col_host
        uu, pp, nn = u.numpy(), p.numpy(), n.numpy()
        for k in range(0, len(uu), 97):
            row = col[rp[uu[k]]:rp[uu[k] + 1]] - g.n_users
            assert pp[k] in row and nn[k] not in row
        # thread count does not change the draw
        u1, p1, n1 = sample_epoch_capped(g, 3 * 30_000, cap, seed=9, shard=shard,
                                         n_shards=n_shards, n_threads=1)
        assert torch.equal(u1, u) and torch.equal(p1, p) and torch.equal(n1, n)


def test_mf_host_grad_adam_equals_fused_host_step(golden):
    """mirec_cpu_bpr_grad + mirec_cpu_adam (HostDataParallel's halves) are
    bitwise mirec_cpu_bpr_step; grad_scale multiplies the gradient only."""
    from furusato_recommend_amd import MF
    f = golden("mf_d32.npz")
    cfg = {"latent_dim_rec": 32, "lr": float(f["lr"]), "decay": float(f["decay"]),
           "device": "cpu", "bpr_batch_size": 64}
    ds = _DS(f["train_user"], f["train_item"], f["n_users"], f["m_items"])
    a, b = MF(cfg, ds), MF(cfg, ds)
    t = torch.from_numpy(f["triples"])
    for m in (a, b):
        m.load_table(torch.from_numpy(f["user_w0"]), torch.from_numpy(f["item_w0"]))
    for _ in range(3):
        la = a.stageOne(t[:, 0], t[:, 1], t[:, 2])
        lb = b.host_grad(t[:, 0], t[:, 1], t[:, 2])
        b.host_adam()
        assert float(la) == float(lb)
        assert torch.equal(a._table, b._table)
        assert torch.equal(a.optim.exp_avg_sq, b.optim.exp_avg_sq)
    g1 = b.host_grad(t[:, 0], t[:, 1], t[:, 2]).clone()
    full = b.host_grad_buffer.clone()
    b.host_grad(t[:, 0], t[:, 1], t[:, 2], grad_scale=0.5)
    assert torch.allclose(b.host_grad_buffer, 0.5 * full, rtol=1e-6, atol=0)
    assert float(g1) == float(b.host_grad(t[:, 0], t[:, 1], t[:, 2]))


def test_train_dp_cli_mf_cpu_registry_two_ranks(golden, tmp_path):
    """``train_dp --model mf --device cpu --gpus 2`` through the model
    registry (no --factory): the host capped sampler, the host
    data-parallel step (gradients all-reduced over gloo), rank-0 evaluation
    and the checkpoint — no HIP call anywhere."""
    import json
    import subprocess
    import sys
    from tests.conftest import ROOT
    _write_split(golden, tmp_path / "data")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    env["HIP_VISIBLE_DEVICES"] = ""  # a host without a GPU
    ck = tmp_path / "ck"
    cmd = [sys.executable, "-m", "furusato_recommend_amd.train_dp", "--model", "mf",
           "--gpus", "2", "--device", "cpu", "--data", str(tmp_path / "data"),
           "--recdim", "16", "--bpr_batch", "16", "--test_span", "1", "--epochs", "2",
           "--path", str(ck)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert [x["epoch"] for x in recs] == [0, 1] and recs[0]["world"] == 2
    assert recs[0]["triples_per_rank"] > 0 and all(np.isfinite(x["loss"]) for x in recs)
    assert recs[1]["loss"] < recs[0]["loss"] + 1e-3
    for k in ("recall", "ndcg"):
        assert all(np.isfinite(recs[1]["metrics"][k]))
    assert (ck / "ddp_mf_all.pth").exists()
