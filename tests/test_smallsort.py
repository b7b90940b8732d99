"""The library's own sort of up to 8 192 pairs (mirec_small_sort_pairs,
csrc/smallsort.hip: the BPR seed grouping) against numpy's stable argsort —
keys and values at every 256-entry chunk edge, duplicate-heavy and
single-key inputs, explicit values, sentinel keys, replays of a captured HIP
graph; n above the bound is refused."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sort(keys, vals=None):
    from furusato_recommend_amd import _lib
    from furusato_recommend_amd._lib import check, lib
    kt = torch.from_numpy(keys.astype(np.int32)).cuda()
    vt = None if vals is None else torch.from_numpy(vals.astype(np.int32)).cuda()
    ko, vo = torch.empty_like(kt), torch.empty_like(kt)
    nb = ctypes.c_size_t()
    check(lib.mirec_small_sort_workspace(kt.numel(), ctypes.byref(nb)))
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device="cuda")
    check(lib.mirec_small_sort_pairs(kt.data_ptr(), vt.data_ptr() if vt is not None else None,
                                     ko.data_ptr(), vo.data_ptr(), kt.numel(), ws.data_ptr(),
                                     nb.value, _lib.stream_handle()))
    return ko.cpu().numpy(), vo.cpu().numpy()


@pytest.mark.parametrize("n", [1, 2, 3, 7, 255, 256, 257, 1000, 6144, 8191, 8192])
@pytest.mark.parametrize("kind", ["wide", "dups", "one"])
def test_small_sort_is_the_stable_order(n, kind):
    rng = np.random.default_rng(n)
    if kind == "wide":
        keys = rng.integers(0, 1_100_001, n)
    elif kind == "dups":
        keys = rng.integers(0, max(1, n // 20), n) * 37
    else:
        keys = np.full(n, 100_000)
    ko, vo = _sort(keys)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ko, keys[order])
    assert np.array_equal(vo, order)


def test_small_sort_values_and_sentinels():
    rng = np.random.default_rng(1)
    n = 8000
    keys = rng.integers(0, 300, n)
    keys[rng.random(n) < 0.3] = 100_000  # a sentinel bucket (invalid ids sort last)
    vals = rng.integers(-2 ** 31, 2 ** 31 - 1, n)
    ko, vo = _sort(keys, vals)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ko, keys[order]) and np.array_equal(vo, vals[order])


def test_small_sort_refuses_above_bound():
    from furusato_recommend_amd._lib import lib
    assert lib.mirec_small_sort_workspace(8193, ctypes.byref(ctypes.c_size_t())) != 0


@pytest.mark.parametrize("n", [6144, 8192])
def test_small_sort_graph_replay(n):
    from furusato_recommend_amd import _lib
    from furusato_recommend_amd._lib import check, lib
    kt = torch.zeros(n, dtype=torch.int32, device="cuda")
    ko, vo = torch.empty_like(kt), torch.empty_like(kt)
    nb = ctypes.c_size_t()
    check(lib.mirec_small_sort_workspace(n, ctypes.byref(nb)))
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            check(lib.mirec_small_sort_pairs(kt.data_ptr(), None, ko.data_ptr(), vo.data_ptr(), n,
                                             ws.data_ptr(), nb.value, _lib.stream_handle()))
    rng = np.random.default_rng(n)
    for it in range(3):
        keys = rng.integers(0, 100_001 if it else 50, n)
        kt.copy_(torch.from_numpy(keys.astype(np.int32)))
        g.replay()
        torch.cuda.synchronize()
        order = np.argsort(keys, kind="stable")
        assert np.array_equal(ko.cpu().numpy(), keys[order]), it
        assert np.array_equal(vo.cpu().numpy(), order), it
