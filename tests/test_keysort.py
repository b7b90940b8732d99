"""The counting sort of dense keys (mirec_key_sort_pairs, csrc/keysort.hip)
against numpy's stable argsort: keys, values and bucket starts identical,
over the bucket classes the kernel treats differently (small <= 32 entries,
mid <= mid_max, big above it), skewed (hub) and sentinel-heavy key sets,
ragged sizes, reruns bitwise and a captured HIP-graph replay."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _keys(kind, n, nk, rng):
    return np.minimum(_keys_raw(kind, n, nk, rng), nk - 1).astype(np.int64)


def _keys_raw(kind, n, nk, rng):
    if kind == "uniform":
        return rng.integers(0, nk, n)
    if kind == "zipf":   # a few hub ids with 10^4-10^5 entries, a long tail
        return np.minimum(rng.zipf(1.3, n) - 1, nk - 1)
    if kind == "one":    # every entry in one bucket (big)
        return np.full(n, nk // 2)
    if kind == "mid":    # ~n/300 buckets of ~300 entries (mid class)
        return rng.integers(0, max(1, n // 300), n) * 7 % nk
    if kind == "sentinel":  # half the entries in the last bucket (invalid ids)
        k = rng.integers(0, max(1, nk - 1), n)
        k[rng.random(n) < 0.5] = nk - 1
        return k
    if kind == "mixed":  # small, mid and big buckets side by side
        parts = [rng.integers(0, nk, n // 2), np.full(n // 8, 3), np.full(n // 8, nk - 2),
                 rng.integers(10, 10 + max(1, n // 500), n - n // 2 - 2 * (n // 8))]
        k = np.concatenate(parts)
        rng.shuffle(k)
        return k
    raise ValueError(kind)


def _check(keys, nk, vals=None):
    from furusato_recommend_amd.rows import key_sort_pairs
    kt = torch.from_numpy(keys.astype(np.int32)).cuda()
    vt = None if vals is None else torch.from_numpy(vals.astype(np.int32)).cuda()
    ko, vo, off = key_sort_pairs(kt, nk, vt, offsets=True)
    order = np.argsort(keys, kind="stable")
    want_v = order if vals is None else vals[order]
    assert np.array_equal(ko.cpu().numpy(), keys[order])
    assert np.array_equal(vo.cpu().numpy(), want_v)
    want_off = np.concatenate([[0], np.cumsum(np.bincount(keys, minlength=nk))])
    assert np.array_equal(off.cpu().numpy(), want_off)
    return ko, vo


@pytest.mark.parametrize("kind", ["uniform", "zipf", "one", "mid", "sentinel", "mixed"])
@pytest.mark.parametrize("n,nk", [(1_757_184, 1_100_001), (63_488, 100_001), (6144, 1_100_000),
                                  (1, 1), (33, 5), (5000, 3), (300_001, 8193)])
def test_key_sort_matches_stable_argsort(kind, n, nk):
    rng = np.random.default_rng(n + nk)
    keys = _keys(kind, n, nk, rng)
    _check(keys, nk)


def test_key_sort_values_and_reruns_bitwise():
    rng = np.random.default_rng(5)
    n, nk = 400_000, 50_000
    keys = _keys("mixed", n, nk, rng)
    vals = rng.integers(-2**31, 2**31 - 1, n)
    a = _check(keys, nk, vals)
    b = _check(keys, nk, vals)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_key_sort_large_n_big_tiles():
    """n above 4 M: tiles grow past 4096 entries and mid_max past 1024."""
    rng = np.random.default_rng(9)
    n, nk = 20_000_000, 2_000_000
    keys = _keys("mixed", n, nk, rng)
    _check(keys, nk)


def test_key_sort_out_of_range_keys_go_last():
    rng = np.random.default_rng(3)
    nk = 1000
    keys = rng.integers(-5, nk + 5, 20_000)
    from furusato_recommend_amd.rows import key_sort_pairs
    ko, vo = key_sort_pairs(torch.from_numpy(keys.astype(np.int32)).cuda(), nk)
    clamped = np.where((keys >= 0) & (keys < nk), keys, nk - 1)
    order = np.argsort(clamped, kind="stable")
    assert np.array_equal(ko.cpu().numpy(), clamped[order])
    assert np.array_equal(vo.cpu().numpy(), order)


def test_key_sort_graph_replay():
    """Captured once, replayed on new keys written into the same buffer."""
    import ctypes

    from furusato_recommend_amd import _lib
    from furusato_recommend_amd._lib import check, lib
    n, nk = 70_000, 20_000
    rng = np.random.default_rng(11)
    kt = torch.zeros(n, dtype=torch.int32, device="cuda")
    ko = torch.empty_like(kt)
    vo = torch.empty_like(kt)
    nb = ctypes.c_size_t()
    check(lib.mirec_key_sort_workspace(n, nk, ctypes.byref(nb)))
    ws = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            check(lib.mirec_key_sort_pairs(kt.data_ptr(), None, ko.data_ptr(), vo.data_ptr(), None,
                                           n, nk, ws.data_ptr(), nb.value,
                                           _lib.stream_handle()))
    for kind in ["zipf", "uniform", "mixed", "one"]:
        keys = _keys(kind, n, nk, rng)
        kt.copy_(torch.from_numpy(keys.astype(np.int32)))
        g.replay()
        torch.cuda.synchronize()
        order = np.argsort(keys, kind="stable")
        assert np.array_equal(ko.cpu().numpy(), keys[order]), kind
        assert np.array_equal(vo.cpu().numpy(), order), kind
