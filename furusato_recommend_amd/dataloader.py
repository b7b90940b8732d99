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


class Loader(_Base):
    """Text-file loader with dataloader.py:73-173 semantics."""

    def __init__(self, config: dict | None = None, path: str = "./data/cf"):
        super().__init__()
        config = config or {}
        suffix = config.get("suffix", "")
        test_mode = bool(config.get("test", False))
        train_file = os.path.join(path, suffix, f"train{suffix}.txt")
        test_file = os.path.join(path, suffix, f"test{suffix}.txt")
        tu, ti, allpos = [], [], []
        self.n_user = 0
        self.m_item = 0
        with open(train_file) as f:
            for line in f:
                parts = line.strip("\n").split(" ")
                if len(parts) < 1 or parts[0] == "":
                    continue
                uid = int(parts[0])
                items = [int(x) for x in parts[1:] if x != ""]
                tu.extend([uid] * len(items))
                ti.extend(items)
                allpos.append(np.array(items, dtype=np.int64))
                if items:
                    self.m_item = max(self.m_item, max(items))
                self.n_user = max(self.n_user, uid)
                if uid == 100 and test_mode:
                    break
        test_u, test_i = [], []
        if os.path.exists(test_file):
            with open(test_file) as f:
                for line in f:
                    parts = line.strip("\n").split(" ")
                    if len(parts) < 1 or parts[0] == "":
                        continue
                    uid = int(parts[0])
                    items = [int(x) for x in parts[1:] if x != ""]
                    test_u.extend([uid] * len(items))
                    test_i.extend(items)
                    if items:
                        self.m_item = max(self.m_item, max(items))
                    self.n_user = max(self.n_user, uid)
                    if uid == 100 and test_mode:
                        break
        self.m_item += 1
        self.n_user += 1
        self.trainUser = np.array(tu, dtype=np.int64)
        self.trainItem = np.array(ti, dtype=np.int64)
        self._allPos = allpos  # indexed by train-file line, as the reference
        self.testUser = np.array(test_u, dtype=np.int64)
        self.testItem = np.array(test_i, dtype=np.int64)
        self._testDict = {}
        for u, i in zip(test_u, test_i):
            self._testDict.setdefault(u, []).append(i)


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
