"""Model plugin for the train_dp launcher's CPU test (``--factory
tests.dp_cli_factory:make``): LightGCN over the CPU oracle (test
infrastructure, never the product path) behind the real
``dist.DataParallel``, with a rank-shard sampler and the oracle's
evaluation, so the launcher's whole process tree (torch.distributed.run,
gloo rendezvous, DPTrainer epochs, evaluation, checkpoint, resume) runs
without a GPU."""
import numpy as np
import torch

from oracle import lightgcn_oracle as O
from tests.test_host import _AccumEngine, _CpuLGCN, _dp_sampler


def make(config, dataset, rank, world):
    from furusato_recommend_amd.dist import DataParallel
    tu = np.asarray(dataset.trainUser, np.int64)
    ti = np.asarray(dataset.trainItem, np.int64)
    nu, mi = int(dataset.n_users), int(dataset.m_items)
    g = torch.Generator().manual_seed(int(config["seed"]) + 31 * rank)  # rank 1: overwritten
    emb = torch.randn(nu + mi, int(config["recdim"]), generator=g) * 0.1
    o = O.OracleLightGCN(tu, ti, nu, mi, int(config["recdim"]), int(config["layer"]),
                         float(config["lr"]), float(config["decay"]), emb=emb)
    model = _CpuLGCN(o)
    dp = DataParallel(_AccumEngine(o, int(config["bpr_batch_size"])), o.emb.data, o.optim,
                      mode="sparse")
    pos = [set() for _ in range(nu)]
    for u, i in zip(tu.tolist(), ti.tolist()):
        pos[u].add(i)
    test = dataset.testDict

    def evaluator(m):
        with torch.no_grad():
            out = m.o.propagated()
        ue, ie = out[:nu], out[nu:]
        allpos = [np.array(sorted(s)) for s in pos]
        res = O.evaluate(ue, ie, test, allpos, topks=tuple(config["topks"]))
        users = sorted(test)
        r = ue[torch.tensor(users)] @ ie.t()
        for k, u in enumerate(users):
            r[k, list(pos[u])] = -(1 << 10)
        return res, torch.topk(r, max(config["topks"])).indices.numpy()
    return {"model": model, "dp": dp, "sampler": _dp_sampler(pos, nu, mi, rank, world),
            "evaluator": evaluator}
