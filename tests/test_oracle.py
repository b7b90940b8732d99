"""The CPU oracle pinned against fixtures generated from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import lightgcn_oracle as O
from tests.conftest import GOLDEN

LGCN = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "lgcn_*.npz")))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("name", LGCN)
def test_forward_matches_reference(golden, name):
    f = golden(name)
    n_users, L = int(f["n_users"]), int(f["n_layers"])
    ei = O.edge_index(f["train_user"], f["train_item"], n_users)
    out, layers = O.forward(torch.from_numpy(f["emb0"]), ei, n_users, L, return_layers=True)
    assert rel(out, f["out_radj"]) < 1e-6          # reference's own formula
    assert rel(out, f["out"]) < 1e-5               # LGConv (gcn_norm) path
    for l in range(L + 1):
        assert rel(layers[l], f["layers"][l]) < 1e-5
    # The two reference formulations (rAdjConv r=.5 vs LGConv) agree.
    assert rel(f["out"], f["out_radj"]) < 1e-5


@pytest.mark.parametrize("name", LGCN)
def test_loss_grad_and_adam_match_reference(golden, name):
    f = golden(name)
    n_users, m_items = int(f["n_users"]), int(f["m_items"])
    m = O.OracleLightGCN(f["train_user"], f["train_item"], n_users, m_items, int(f["dim"]),
                         int(f["n_layers"]), float(f["lr"]), float(f["decay"]),
                         emb=torch.from_numpy(f["emb0"]))
    t = f["triples"]
    loss, reg = m.bpr_loss(t[:, 0], t[:, 1], t[:, 2])
    assert abs(float(loss) - float(f["loss"])) < 1e-6
    assert abs(float(reg) - float(f["reg"])) / float(f["reg"]) < 1e-6
    g = m.grad(t[:, 0], t[:, 1], t[:, 2])
    assert rel(g, f["grad"]) < 1e-5
    l1 = m.stageOne(t[:, 0], t[:, 1], t[:, 2])
    assert rel(m.emb.detach(), f["emb_step1"]) < 2e-5
    l2 = m.stageOne(t[:, 0], t[:, 1], t[:, 2])
    assert rel(m.emb.detach(), f["emb_step2"]) < 2e-5
    assert np.allclose([l1, l2], f["step_losses"], rtol=1e-6)


def test_mf_matches_reference(golden):
    f = golden("mf_d32.npz")
    m = O.OracleMF(torch.from_numpy(f["user_w0"]), torch.from_numpy(f["item_w0"]),
                   float(f["lr"]), float(f["decay"]))
    t = f["triples"]
    loss, reg = m.bpr_loss(t[:, 0], t[:, 1], t[:, 2])
    assert abs(float(loss) - float(f["loss"])) < 1e-5
    assert abs(float(reg) - float(f["reg"])) / float(f["reg"]) < 1e-6
    sl = m.stageOne(t[:, 0], t[:, 1], t[:, 2])
    assert abs(sl - float(f["step_loss"])) < 1e-5
    assert rel(m.user.detach(), f["user_w1"]) < 1e-6
    assert rel(m.item.detach(), f["item_w1"]) < 1e-6


def test_sampler_bit_exact(golden):
    f = golden("sampler.npz")
    u, i = f["train_user"], f["train_item"]
    n_users, m_items = int(f["n_users"]), int(f["m_items"])
    all_pos = [i[u == k] for k in range(n_users)]
    np.random.seed(int(f["seed"]))
    S = O.uniform_sample(n_users, m_items, all_pos, len(u))
    assert np.array_equal(S, f["S"])
    for uu, p, n in S:  # the sampler's own invariants
        assert p in all_pos[uu] and n not in all_pos[uu]


def _weighted_probs(f):
    u, i, n_users = f["train_user"], f["train_item"], int(f["n_users"])
    all_pos = [i[u == k] for k in range(n_users)]
    flat, probs, o = f["probs_flat"], [], 0
    for pu in all_pos:
        probs.append(flat[o:o + len(pu)])
        o += len(pu)
    assert o == len(flat)
    return all_pos, probs


def test_weighted_sampler_bit_exact(golden):
    """oracle.weighted_sample == the reference's UniformSampling.sample_parallel
    with per-user probabilities (negative_sample.py:45-72, sample_pow != 0),
    draw for draw; zero-probability positives never drawn."""
    f = golden("sampler_weighted.npz")
    all_pos, probs = _weighted_probs(f)
    np.random.seed(int(f["seed"]))
    S = O.weighted_sample(int(f["n_users"]), int(f["m_items"]), all_pos, len(f["train_user"]),
                          probs)
    assert np.array_equal(S, f["S"])
    for uu, p, n in S:
        pu, pr = all_pos[uu], probs[uu]
        assert pr[pu == p].sum() > 0 and n not in pu


def test_metrics_match_reference(golden):
    f = golden("metrics.npz")
    gt = np.split(f["gt_flat"], np.cumsum(f["gt_len"])[:-1])
    gt = [list(g) for g in gt]
    r = O.get_label(gt, f["pred"])
    assert np.array_equal(r, f["label"])
    for k in (10, 20):
        ret = O.recall_precision_at_k(gt, r, k)
        assert np.isclose(ret["recall"], f[f"recall_at_{k}"])
        assert np.isclose(ret["precision"], f[f"precision_at_{k}"])
        assert ret["hr"] == f[f"hr_at_{k}"]
        assert np.isclose(O.ndcg_at_k(gt, r, k), f[f"ndcg_at_{k}"])


def sage_groups(f):
    return np.split(f["groups"], np.cumsum(f["group_len"])[:-1])


SAGE = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "sage_*.npz")))


@pytest.mark.parametrize("name", SAGE)
def test_sage_matches_reference(golden, name):
    """The tree restatement of GraphSAGE.forward / loss == the reference's
    own forward on the equivalent PyG adjacency (model/graphsage.py:311-337)."""
    f = golden(name)
    L, sizes, d = int(f["n_layers"]), [int(x) for x in f["sizes"]], int(f["dim"])
    nu = int(f["n_users"])
    table = torch.nn.Parameter(torch.from_numpy(f["table0"]).clone())
    lins = torch.nn.ModuleList([torch.nn.Linear(2 * d, d) for _ in range(L)])
    with torch.no_grad():
        for k, li in enumerate(lins):
            li.weight.copy_(torch.from_numpy(f[f"w{k}"]))
            li.bias.copy_(torch.from_numpy(f[f"b{k}"]))
    depths, _ = O.sage_canonical_layout(L)
    assert list(f["group_depth"]) == depths
    out = O.sage_forward(table, lins, sage_groups(f), L, sizes)
    B = int(f["batch"])
    assert rel(out.detach(), f["emb_out"][:3 * B]) < 1e-6
    reg = [table[:nu], table[nu:]] + [p for li in lins for p in (li.weight, li.bias)]
    loss = O.sage_loss(out[:B], out[B:2 * B], out[2 * B:], reg, float(f["decay"]))
    assert abs(float(loss) - float(f["loss"])) < 1e-6
    loss.backward()
    assert rel(table.grad, f["g_table"]) < 1e-5
    for k, li in enumerate(lins):
        assert rel(li.weight.grad, f[f"g_w{k}"]) < 1e-5
        assert rel(li.bias.grad, f[f"g_b{k}"]) < 1e-5


@pytest.mark.parametrize("name", ["sasrec_d64_h8.npz", "sasrec_d128_h2.npz"])
def test_sasrec_block_matches_reference(golden, name):
    """Written-out causal MHA + block + masked mean == the reference's
    SASRec.forward_user over torch.nn.MultiheadAttention (dropout off)."""
    f = golden(name)
    L, heads = int(f["L"]), int(f["heads"])
    p = {k: torch.from_numpy(v).requires_grad_(True) for k, v in f.items()
         if not k.startswith("g_") and k not in ("d", "heads", "L", "lengths", "x", "out", "wts")}
    x = torch.from_numpy(f["x"]).requires_grad_(True)
    out = O.sasrec_forward_user(x, f["lengths"], p, heads, L)
    assert rel(out.detach(), f["out"]) < 1e-5
    (out * torch.from_numpy(f["wts"])).sum().backward()
    assert rel(x.grad, f["g_x"]) < 1e-5
    for k, v in p.items():
        assert rel(v.grad, f["g_" + k]) < 1e-4, k


GRAPH_CASES = [("sym", 16), ("sym", 48), ("dir", 64), ("dir", 256)]


def lgconv_case(f, name, d):
    """(edge_index, x, y, ybar, xbar, y_sum or None) of one LGConv fixture;
    the cotangent ybar is regenerated from its seed (make_golden.py)."""
    n = int(f[f"{name}_n"])
    ybar = torch.randn(n, d, generator=torch.Generator().manual_seed(2000 + d))
    return (torch.from_numpy(f[f"{name}_edge_index"]), torch.from_numpy(f[f"{name}_d{d}_x"]),
            f[f"{name}_d{d}_y"], ybar, f[f"{name}_d{d}_xbar"], f.get(f"{name}_d{d}_y_sum"))


@pytest.mark.parametrize("name,d", GRAPH_CASES)
def test_pyg_lgconv_matches_fixture(golden, name, d):
    """Non-bipartite / directed graphs (PyG LGConv semantics)."""
    f = golden("lgconv_graphs.npz")
    ei, x, y, ybar, xbar, ysum = lgconv_case(f, name, d)
    xr = x.clone().requires_grad_(True)
    yo = O.pyg_lgconv(xr, ei)
    assert rel(yo.detach(), y) < 1e-6
    (yo * ybar).sum().backward()
    assert rel(xr.grad, xbar) < 1e-6
    if ysum is not None:
        assert rel(O.pyg_lgconv(x, ei, normalize=False), ysum) < 1e-6
    # symmetric graphs: PyG's gcn_norm equals the reference's own rAdjConv
    # formula (model/radj.py:28-44, source-degree r = 0.5)
    if name == "sym":
        assert rel(O.lgconv(x, ei), y) < 1e-5
