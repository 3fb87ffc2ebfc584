"""GPU parity of the bounded wide scan (ivf_scan_bounded): wide items of many queries
are bounded on the matrix cores and only candidates that can reach the top-k are
recomputed with the reference's sequential fp32 sum (search_list_cpu,
ivf_flat_index.cpp:347-370). Results must stay bit-identical to the oracle whatever
the bound prunes, so these cases stress the pruning rules: hub lists probed by every
query, k around the block-bound limit (16), both metrics, a cancellation regime where
the bound is wider than the whole distance spread (every pair a candidate), ties,
duplicate ids and infinite / overflowing values.
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb

vdb = load_vdb()
pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_same(D, I, Dr, Ir):
    bad = np.argwhere(I != Ir)
    assert bad.size == 0, f"ids differ at {bad[:5].tolist()}: gpu {I[tuple(bad[0])]} ref {Ir[tuple(bad[0])]}"
    badd = np.argwhere(bits(D) != bits(Dr))
    assert badd.size == 0, f"dist bits differ at {badd[:5].tolist()}: gpu {D[tuple(badd[0])]!r} ref {Dr[tuple(badd[0])]!r}"


def lists_pair(X, ids, lists, C, metric):
    """Engine + oracle with the given centroids and explicit list assignment."""
    import torch
    dim, nlist = X.shape[1], C.shape[0]
    o = oracle.OracleIndex(dim, nlist, metric)
    o.centroids = C
    for l in range(nlist):
        m = lists == l
        o.set_list(l, X[m], ids[m])
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, vdb.Metric(metric)))
    g.centroids = C
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
    idd = torch.from_numpy(ids.view(np.int64)).to(dev)
    ld = torch.from_numpy(lists.astype(np.int32)).to(dev)
    # the oracle's list order is list-major in input order: add in the same order
    g.add_to_lists_device(xd.data_ptr(), idd.data_ptr(), ld.data_ptr(), len(X))
    torch.cuda.synchronize()
    for l in range(nlist):
        assert np.array_equal(g.get_list(l)[1], o.get_list(l)[1])
    return g, o


def hub_data(dim, seed, n_hub=30000, n_other=2000, nlist=6):
    rng = np.random.default_rng(seed)
    n = n_hub + n_other * (nlist - 1)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    lists = np.concatenate([np.zeros(n_hub, np.int64)] + [np.full(n_other, l) for l in range(1, nlist)])
    perm = rng.permutation(n)
    X, lists = X[perm], lists[perm]
    ids = rng.permutation(n).astype(np.uint64)
    C = np.zeros((nlist, dim), np.float32)
    C[1:] = 3.0 * rng.standard_normal((nlist - 1, dim)).astype(np.float32)
    Q = rng.standard_normal((130, dim)).astype(np.float32)
    return X, ids, lists, C, Q


def search_all(g, Q, nprobe, k, batch):
    g.set_batch(batch)
    return g.search(Q, nprobe=nprobe, k=k)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [1, 10, 16, 17, 64])
def test_bounded_hub_lists(metric, k):
    X, ids, lists, C, Q = hub_data(48, seed=3 + k)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen", 0)  # (the bounded scan serves only with the screen off)
    nprobe = 3 if metric == 0 else 6  # IP: every list (the origin centroid ties at 0)
    Dr, Ir = o.search(Q, nprobe, k)
    for mm in (1, 8, 0):  # every wide item bounded / items of >= 8 queries / never (the default)
        g.set_option("scan_mfma_min", mm)
        for batch in (64, 130):
            for seg, spi in ((0, 0), (64, 12)):
                g.set_option("seg_vectors", seg)
                g.set_option("segs_per_item", spi)
                assert_same(*search_all(g, Q, nprobe, k, batch), Dr, Ir)
    g.set_option("scan_mfma_min", 0)


def test_bounded_path_is_taken_and_prunes():
    X, ids, lists, C, Q = hub_data(64, seed=5)
    g, o = lists_pair(X, ids, lists, C, 0)
    g.set_option("screen", 0)  # (the bounded scan serves only with the screen off)
    g.set_option("scan_mfma_min", 1)
    g.set_option("bounded_stats", 1)  # statistics only: results stay valid
    g.profile_reset()
    D, I = search_all(g, Q, 3, 10, 130)
    p = g.profile_read()
    g.set_option("bounded_stats", 0)
    assert_same(D, I, *o.search(Q, 3, 10))
    assert p["bounded_blocks"] > 0, p
    # every query scans the 30000-vector hub list: iid data prunes most pairs
    assert 0 < p["exact_reranks"] < 0.5 * p["pair_vectors"], p
    print("bounded stats", p)


@pytest.mark.parametrize("metric", [0, 1])
def test_bounded_cancellation_every_pair_a_candidate(metric):
    """Vectors and queries in a tiny ball far from the origin: |q|, |x| ~ 100 while
    distances ~ 1e-2, so the bound (~ 1e-4 (|q| + |x|)^2) exceeds the whole distance
    spread and every pair goes through the exact re-rank (full candidate lists)."""
    rng = np.random.default_rng(11)
    dim = 40
    c = (100.0 / np.sqrt(dim)) * np.ones(dim, np.float32)
    X = (c + 0.01 * rng.standard_normal((12000, dim))).astype(np.float32)
    Q = (c + 0.01 * rng.standard_normal((96, dim))).astype(np.float32)
    lists = (rng.random(12000) >= 0.8).astype(np.int64)
    ids = np.arange(12000, dtype=np.uint64)
    C = np.stack([c, -c]).astype(np.float32)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen", 0)  # (the bounded scan serves only with the screen off)
    Dr, Ir = o.search(Q, 2, 10)
    g.set_option("scan_mfma_min", 1)
    g.set_option("bounded_stats", 1)
    g.profile_reset()
    D, I = search_all(g, Q, 2, 10, 96)
    p = g.profile_read()
    g.set_option("bounded_stats", 0)
    g.set_option("scan_mfma_min", 0)
    assert_same(D, I, Dr, Ir)
    if metric == 0:  # (IP: -<q, x> ~ -1e4 spreads by ~6, wider than its bound; pruning still works)
        assert p["exact_reranks"] > 0.5 * p["pair_vectors"], p


def test_bounded_ties_duplicates_nonfinite():
    rng = np.random.default_rng(17)
    dim = 32
    base = rng.standard_normal((3000, dim)).astype(np.float32)
    X = np.concatenate([base, base, base[:500]])           # exact duplicate vectors: equal distances
    ids = np.concatenate([np.arange(3000), np.arange(3000) + 10000, np.arange(500)]).astype(np.uint64)  # dup ids
    # (no NaN: the reference ranks with std::partial_sort on (dist, id) pairs, and a NaN
    # key breaks its strict weak order, so where it lands is undefined behaviour)
    X[17, 3] = np.inf
    X[31, :] = -np.inf
    X[40, 5] = 3.0e38                                      # finite, overflows when squared
    lists = np.zeros(len(X), np.int64)
    lists[rng.random(len(X)) < 0.1] = 1
    C = np.zeros((2, dim), np.float32)
    C[1] = 5.0
    g, o = lists_pair(X, ids, lists, C, 0)
    g.set_option("screen", 0)  # (the bounded scan serves only with the screen off)
    Q = np.concatenate([base[:48] + 1e-3 * rng.standard_normal((48, dim)).astype(np.float32),
                        rng.standard_normal((40, dim)).astype(np.float32)])
    for k in (5, 10, 40):
        Dr, Ir = o.search(Q, 2, k)
        for mm in (1, 0):
            g.set_option("scan_mfma_min", mm)
            assert_same(*search_all(g, Q, 2, k, 88), Dr, Ir)
    g.set_option("scan_mfma_min", 0)


@pytest.mark.parametrize("dim", [1, 3, 67, 130])
def test_bounded_odd_dimensions(dim):
    X, ids, lists, C, Q = hub_data(dim, seed=dim, n_hub=12000, n_other=800)
    g, o = lists_pair(X, ids, lists, C, 0)
    g.set_option("screen", 0)  # (the bounded scan serves only with the screen off)
    g.set_option("scan_mfma_min", 1)
    assert_same(*search_all(g, Q, 3, 10, 130), *o.search(Q, 3, 10))
    g.set_option("scan_mfma_min", 0)
