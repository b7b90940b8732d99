"""Datasets with the reference's Loader protocol (dataloader.py:66-297).

Protocol used by the models / trainer / samplers: ``n_users``, ``m_items``,
``trainUser``, ``trainItem`` (int64 arrays, one entry per interaction),
``trainDataSize``, ``allPos`` (list indexed by user of that user's train
items, in file order), ``testDict`` ({user: [items]}) and
``getUserPosItems(users)``.

``Loader`` parses the reference's ``train{suffix}.txt`` / ``test{suffix}.txt``
files (``uid i1 i2 ...`` per line, dataloader.py:93-150).
``SyntheticBipartite`` generates the BASELINE configs without
files: every uid has at least one train edge and uids are contiguous, which
the reference's line-indexed ``allPos`` requires (dataloader.py:118,
negative_sample.py:115).
"""
from __future__ import annotations

import os

import numpy as np
import torch


class _Base:
    def __init__(self):
        self._allPos = None

    @property
    def n_users(self) -> int:
        return self.n_user

    @property
    def m_items(self) -> int:
        return self.m_item

    @property
    def trainDataSize(self) -> int:
        return int(self.trainUser.shape[0])

    @property
    def testDict(self) -> dict:
        return self._testDict

    @property
    def allPos(self) -> list:
        if self._allPos is None:
            order = np.argsort(self.trainUser, kind="stable")
            items = self.trainItem[order]
            counts = np.bincount(self.trainUser, minlength=self.n_user)
            self._allPos = np.split(items, np.cumsum(counts)[:-1])
        return self._allPos

    def getUserPosItems(self, users):
        return [self.allPos[int(u)] for u in users]


def parse_interactions(path: str, stop_uid: int = -1, n_threads: int | None = None):
    """Native parse of a ``uid i1 i2 ...`` file (mirec_parse_interactions):
    (line_uid [L], line_off [L+1], items [I], max_uid, max_item), file order."""
    import ctypes

    from ._lib import check, lib
    data = np.fromfile(path, dtype=np.uint8)
    nt = int(n_threads or min(16, os.cpu_count() or 1))
    L, I = ctypes.c_int64(0), ctypes.c_int64(0)
    mu, mi = ctypes.c_int64(0), ctypes.c_int64(0)
    ptr = data.ctypes.data if data.size else None
    check(lib.mirec_parse_interactions(ptr, data.size, int(stop_uid), nt, ctypes.byref(L),
                                       ctypes.byref(I), ctypes.byref(mu), ctypes.byref(mi),
                                       None, None, None), f"parse {path}")
    line_uid = np.empty(L.value, np.int64)
    line_off = np.empty(L.value + 1, np.int64)
    items = np.empty(I.value, np.int64)
    check(lib.mirec_parse_interactions(ptr, data.size, int(stop_uid), nt, ctypes.byref(L),
                                       ctypes.byref(I), ctypes.byref(mu), ctypes.byref(mi),
                                       line_uid.ctypes.data, line_off.ctypes.data,
                                       items.ctypes.data), f"parse {path}")
    return line_uid, line_off, items, mu.value, mi.value


class _LineIndexed(list):
    """allPos built lazily from the parsed offsets: element k is line k's
    items (a view), as the reference's line-indexed list."""

    def __init__(self, items, off):
        super().__init__()
        self._items, self._off = items, off
        self._n = len(off) - 1

    def _fill(self):
        if self._n and not super().__len__():
            self.extend(np.split(self._items, self._off[1:-1]))

    def __len__(self):
        return self._n

    def __getitem__(self, k):
        if isinstance(k, slice):
            self._fill()
            return super().__getitem__(k)
        k = int(k)
        if k < 0:
            k += self._n
        if not 0 <= k < self._n:
            raise IndexError(k)
        return self._items[self._off[k]:self._off[k + 1]]

    def __iter__(self):
        for k in range(self._n):
            yield self[k]


class Loader(_Base):
    """Text-file loader with dataloader.py:73-173 semantics, parsed by the
    native multi-threaded reader (the reference's Python loop runs ~1e5
    lines/s; tools/bench_ingest.py times both)."""

    def __init__(self, config: dict | None = None, path: str = "./data/cf"):
        super().__init__()
        config = config or {}
        suffix = config.get("suffix", "")
        stop = 100 if bool(config.get("test", False)) else -1
        train_file = os.path.join(path, suffix, f"train{suffix}.txt")
        test_file = os.path.join(path, suffix, f"test{suffix}.txt")
        uid, off, items, mu, mi = parse_interactions(train_file, stop)
        counts = np.diff(off)
        self.trainUser = np.repeat(uid, counts)
        self.trainItem = items
        self._allPos = _LineIndexed(items, off)  # indexed by train-file line
        n_user, m_item = mu, mi
        self._testDict = {}
        self.testUser = np.zeros(0, np.int64)
        self.testItem = np.zeros(0, np.int64)
        if os.path.exists(test_file):
            tu, toff, titems, tmu, tmi = parse_interactions(test_file, stop)
            tcounts = np.diff(toff)
            self.testUser = np.repeat(tu, tcounts)
            self.testItem = titems
            n_user, m_item = max(n_user, tmu), max(m_item, tmi)
            d = self._testDict
            nz = np.nonzero(tcounts)[0]
            tl = titems.tolist()
            for u, a, b in zip(tu[nz].tolist(), toff[nz].tolist(), toff[nz + 1].tolist()):
                d.setdefault(u, []).extend(tl[a:b])
        # the reference starts both maxima at 0 (dataloader.py:80-81, 121-122)
        self.n_user = int(max(n_user, 0)) + 1
        self.m_item = int(max(m_item, 0)) + 1


class SyntheticBipartite(_Base):
    """Synthetic user–item graph of SURVEY §8d.

    ``kind='uniform'``: users = cat(arange(n_users), randint(n_users, E - n_users)),
    items uniform (item degree ≈ Poisson(E/m)); ``kind='zipf'``: item
    popularity ∝ 1/rank^alpha (load-balance stress); ``kind='cluster'``:
    user u and item i belong to community u % n_clusters / i % n_clusters,
    and an edge picks an item of its user's community with probability
    p_in, else a uniform item (a graph with something to learn: Recall@20
    moves far above chance).  Multi-edges are kept.
    ``test_frac`` of the users (with ≥ 2 edges) have their guaranteed edge
    moved to the test split.
    """

    def __init__(self, n_users: int, m_items: int, n_edges: int, seed: int = 0,
                 kind: str = "uniform", alpha: float = 1.0, test_frac: float = 0.1,
                 n_clusters: int = 20, p_in: float = 0.9):
        super().__init__()
        if n_edges < n_users:
            raise ValueError("need n_edges >= n_users (every user has a train edge)")
        g = torch.Generator().manual_seed(seed)
        users = torch.cat([torch.arange(n_users),
                           torch.randint(0, n_users, (n_edges - n_users,), generator=g)])
        if kind == "uniform":
            items = torch.randint(0, m_items, (n_edges,), generator=g)
        elif kind == "zipf":
            w = 1.0 / torch.arange(1, m_items + 1, dtype=torch.float64) ** alpha
            items = torch.multinomial(w, n_edges, replacement=True, generator=g)
        elif kind == "cluster":
            K = int(n_clusters)
            if m_items < K:
                raise ValueError("need m_items >= n_clusters")
            per = (m_items - 1 - torch.arange(K)) // K + 1  # items i with i % K == c
            c = users % K
            r = torch.rand(n_edges, generator=g)
            slot = (torch.rand(n_edges, generator=g) * per[c]).long()
            inside = c + K * slot
            items = torch.where(r < p_in, inside, torch.randint(0, m_items, (n_edges,),
                                                                generator=g))
        else:
            raise ValueError(kind)
        users = users.numpy().astype(np.int64)
        items = items.numpy().astype(np.int64)
        deg = np.bincount(users, minlength=n_users)
        test_mask = np.zeros(n_edges, dtype=bool)
        if test_frac > 0:
            n_test = int(n_users * test_frac)
            rng = np.random.default_rng(seed + 1)
            cand = rng.choice(n_users, size=n_test, replace=False)
            cand = cand[deg[cand] >= 2]
            test_mask[cand] = True  # edge u is user u's guaranteed edge
        # Group by user like the reference's line-per-user train file.
        keep = ~test_mask
        tu, ti = users[keep], items[keep]
        order = np.argsort(tu, kind="stable")
        self.trainUser = tu[order]
        self.trainItem = ti[order]
        self.n_user = int(n_users)
        self.m_item = int(m_items)
        self._testDict = {int(u): [int(items[u])] for u in np.nonzero(test_mask)[0]}


class FiveCore(_Base):
    """Config C1: every user has exactly `per_user` distinct items (5-core,
    README.md:3-6); the last one is the test item."""

    def __init__(self, n_users: int = 10_000, m_items: int = 1_000, per_user: int = 5,
                 seed: int = 0):
        super().__init__()
        rng = np.random.default_rng(seed)
        items = np.stack([rng.choice(m_items, size=per_user, replace=False)
                          for _ in range(n_users)])
        self.n_user, self.m_item = int(n_users), int(m_items)
        self.trainUser = np.repeat(np.arange(n_users, dtype=np.int64), per_user - 1)
        self.trainItem = items[:, :-1].reshape(-1).astype(np.int64)
        self._testDict = {u: [int(items[u, -1])] for u in range(n_users)}
