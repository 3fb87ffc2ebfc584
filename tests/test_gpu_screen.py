"""GPU parity of the screened scan (screen.hip, the default scan for L2 / IP, k <= 64):
every (query, vector) distance is bounded on the matrix cores from a residual shadow of the
lists (int8 with per-vector scales or bf16, chosen by a calibration batch at the build) and
recomputed with the reference's sequential fp32 sum (search_list_cpu,
ivf_flat_index.cpp:347-370) only where it can reach the list's top-k. Results must stay
bit-identical to the oracle whatever the screen prunes, so these cases stress it: hub
lists probed by every query, both metrics, k up to the screen's 64 and just past it (the
exact scan then serves), a cancellation regime where the bound is wider than the whole
distance spread, ties, duplicate ids, infinite / overflowing / huge / subnormal values,
odd dimensions (both operand pipelines), incremental adds (the shadow is rebuilt), the
residency cap, and the screen against the exact scan on a trained index.
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb
from test_gpu_bounded import assert_same, hub_data, lists_pair, search_all

vdb = load_vdb()
pytestmark = pytest.mark.gpu


def screen_stats(g, Q, nprobe, k, batch):
    g.set_option("bounded_stats", 1)  # statistics only: results stay valid
    g.profile_reset()
    D, I = search_all(g, Q, nprobe, k, batch)
    p = g.profile_read()
    g.set_option("bounded_stats", 0)
    return D, I, p


@pytest.mark.parametrize("defer", [1, 0], ids=["deferred", "inline"])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [1, 10, 16, 17, 64, 65])
def test_screen_hub_lists(metric, k, defer):
    X, ids, lists, C, Q = hub_data(48, seed=30 + k)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_defer", defer)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, k)
    for batch in (64, 130):
        for seg in (0, 64, 1024):
            g.set_option("seg_vectors", seg)
            assert_same(*search_all(g, Q, nprobe, k, batch), Dr, Ir)
    # items of up to 32 queries (an item's waves split in two halves; 16 is the default)
    g.set_option("screen_group", 32)
    assert_same(*search_all(g, Q, nprobe, k, 130), Dr, Ir)
    g.set_option("screen_group", 16)
    g.set_option("screen", 0)
    assert_same(*search_all(g, Q, nprobe, k, 130), Dr, Ir)


@pytest.mark.parametrize("defer", [1, 0], ids=["deferred", "inline"])
def test_screen_is_taken_and_prunes(defer):
    X, ids, lists, C, Q = hub_data(64, seed=5)
    g, o = lists_pair(X, ids, lists, C, 0)
    g.set_option("screen_defer", defer)
    D, I, p = screen_stats(g, Q, 3, 10, 130)
    print("screen stats", p)
    assert_same(D, I, *o.search(Q, 3, 10))
    assert p["bounded_blocks"] > 0, p
    # every query scans the 30000-vector hub list: iid data prunes nearly every pair (round 3
    # measured ~1.7 % re-checked inline; a pruning regression shows up well before 5 %)
    assert 0 < p["exact_reranks"] < 0.05 * p["pair_vectors"], p
    if defer:
        # the deferred scan re-checks only the survivors of each pair's final threshold:
        # far fewer than it collected, and at least k per (query, probed list) pair
        assert p["screen_collected"] >= p["exact_reranks"] >= 10 * len(Q), p
    else:
        assert p["screen_collected"] == 0, p
    g.set_option("screen", 0)
    D, I, p = screen_stats(g, Q, 3, 10, 130)
    assert p["bounded_blocks"] == 0 and p["exact_reranks"] == 0, p


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [1, 10, 17, 64])
def test_screen_int8_shadow_hub_lists(metric, k):
    """The int8 shadow (option screen_i8): per-vector scaled residuals on
    v_mfma_i32_16x16x64_i8, exact integer sums, |b - b'| measured per vector; hub lists,
    16- and 32-query items, several segment sizes; and the format switches back to bf16 for
    the inline kernel and the option 0."""
    X, ids, lists, C, Q = hub_data(48, seed=90 + k)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_i8", 1)
    g.set_option("screen_floor_ppm", 0)  # (at k = 64 the wider bound would trip the floor)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, k)
    for sg in (16, 32):
        g.set_option("screen_group", sg)
        for seg in (0, 64):
            g.set_option("seg_vectors", seg)
            D, I, p = screen_stats(g, Q, nprobe, k, 130)
            assert_same(D, I, Dr, Ir)
            assert p["bounded_blocks"] > 0, p  # (the deferred collect serves every k <= 64 at both widths)
    g.set_option("screen_defer", 0)  # (the inline kernel: a bf16 shadow is built for it)
    assert_same(*search_all(g, Q, nprobe, k, 130), Dr, Ir)
    g.set_option("screen_defer", 1)
    g.set_option("screen_i8", 0)
    assert_same(*search_all(g, Q, nprobe, k, 130), Dr, Ir)


@pytest.mark.parametrize("dim", [1, 3, 67, 130, 256])
def test_screen_int8_odd_dims_and_extremes(dim):
    """int8 shadow with dims that leave 1, 2 or 3 k-steps of 64 (every k-step pipeline),
    plus vectors with huge, infinite and subnormal values and a zero vector."""
    rng = np.random.default_rng(dim)
    X = rng.standard_normal((3000, dim)).astype(np.float32)
    X[5] = 0.0
    X[6, 0] = 3e38
    X[7, 0] = np.inf
    X[8] = 1e-41
    Q = rng.standard_normal((70, dim)).astype(np.float32)
    ids = np.arange(3000, dtype=np.uint64)
    for metric in (0, 1):
        o = oracle.OracleIndex(dim, 8, metric)
        o.centroids = rng.standard_normal((8, dim)).astype(np.float32)
        o.add(X, ids)
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, 8, vdb.Metric(metric)))
        g.centroids = o.centroids
        g.add(X, ids)
        g.set_option("screen_i8", 1)
        for k in (1, 10):
            assert_same(*g.search(Q, nprobe=3, k=k), *o.search(Q, 3, k))


@pytest.mark.parametrize("i8", [1, 0], ids=["int8", "bf16"])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [1, 10, 17, 64])
def test_two_pass_recheck(metric, k, i8):
    """The two-pass exact re-check (ivf_screen_recheck2, default for rows in HBM): per pair
    first the k survivors of smallest lower bound, then only the others whose lower bound is
    not above the k-th exact distance so far. Hub lists probed by every query at 16- and
    32-query items and two segment sizes: results identical to the oracle and to the one-pass
    re-check (screen_recheck2 0), with fewer rows re-checked."""
    X, ids, lists, C, Q = hub_data(64, seed=200 + k)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_i8", i8)
    g.set_option("screen_floor_ppm", 0)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, k)
    for sg in (16, 32):
        g.set_option("screen_group", sg)
        for seg in (0, 64):
            g.set_option("seg_vectors", seg)
            got = {}
            for r2 in (1, 0):
                g.set_option("screen_recheck2", r2)
                D, I, p = screen_stats(g, Q, nprobe, k, 130)
                assert_same(D, I, Dr, Ir)
                got[r2] = p["exact_reranks"]
            assert got[1] <= got[0], got
            if k <= 17:
                assert got[1] < got[0], got
    g.set_option("screen_recheck2", 1)


@pytest.mark.parametrize("metric", [0, 1])
def test_screen_deferred_overflow_recomputes_the_pair(metric):
    """A candidate buffer far too small for the batch: every pair whose candidates do not fit
    is marked and recomputed exactly over its whole list, one wave per planned segment (one
    and several segments per list); results unchanged."""
    X, ids, lists, C, Q = hub_data(48, seed=77)
    g, o = lists_pair(X, ids, lists, C, metric)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, 10)
    g.set_option("screen_cand_cap", 1024)
    g.set_option("screen_floor_ppm", 0)  # (the floor would send the next batches to the exact scan)
    for seg in (64, 0):
        g.set_option("seg_vectors", seg)
        D, I, p = screen_stats(g, Q, nprobe, 10, 130)
        assert_same(D, I, Dr, Ir)
        assert p["screen_collected"] > 1024, p
    g.set_option("screen_cand_cap", 4 << 20)
    assert_same(*search_all(g, Q, nprobe, 10, 130), Dr, Ir)


@pytest.mark.parametrize("defer", [1, 0], ids=["deferred", "inline"])
@pytest.mark.parametrize("metric", [0, 1])
def test_screen_cancellation_every_pair_a_candidate(metric, defer):
    """Vectors and queries in a tiny ball far from the origin (|q|, |x| ~ 100, distances
    ~ 1e-2) stored in lists whose centroids are far from the ball: the residuals are as
    large as the vectors, so the screen's bound exceeds the whole distance spread and
    every pair goes through the exact re-check. (With centroids at the ball the residual
    shadow screens this data well: the second half.)"""
    rng = np.random.default_rng(11)
    dim = 40
    c = (100.0 / np.sqrt(dim)) * np.ones(dim, np.float32)
    X = (c + 0.01 * rng.standard_normal((12000, dim))).astype(np.float32)
    Q = (c + 0.01 * rng.standard_normal((96, dim))).astype(np.float32)
    lists = (rng.random(12000) >= 0.8).astype(np.int64)
    ids = np.arange(12000, dtype=np.uint64)
    C = np.stack([np.zeros_like(c), -c]).astype(np.float32)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_defer", defer)
    Dr, Ir = o.search(Q, 2, 10)
    D, I, p = screen_stats(g, Q, 2, 10, 96)
    assert_same(D, I, Dr, Ir)
    if metric == 0:
        assert p["exact_reranks"] > 0.5 * p["pair_vectors"], p
    C = np.stack([c, c + 0.05]).astype(np.float32)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_defer", defer)
    Dr, Ir = o.search(Q, 2, 10)
    D, I, p = screen_stats(g, Q, 2, 10, 96)
    assert_same(D, I, Dr, Ir)
    if metric == 0:
        assert p["exact_reranks"] < 0.5 * p["pair_vectors"], p


@pytest.mark.parametrize("metric", [0, 1])
def test_screen_run_time_floor(metric):
    """The cancellation regime call after call: a batch whose survivors exceed
    screen_floor_ppm of its pairs trips the floor, and the next screen_floor_skip batches
    run the exact scan; results stay bit-identical through every switch. screen_floor_ppm 0
    never trips."""
    rng = np.random.default_rng(12)
    dim = 48
    c = (100.0 / np.sqrt(dim)) * np.ones(dim, np.float32)
    X = (c + 0.01 * rng.standard_normal((8000, dim))).astype(np.float32)
    Q = (c + 0.01 * rng.standard_normal((6 * 32, dim))).astype(np.float32)
    lists = (rng.random(8000) >= 0.7).astype(np.int64)
    ids = np.arange(8000, dtype=np.uint64)
    C = np.stack([np.zeros_like(c), -c]).astype(np.float32)
    g, o = lists_pair(X, ids, lists, C, metric)
    g.set_option("screen_floor_skip", 3)
    g.set_option("screen_floor_min", 0)  # (these batches are small: 32 x ~5600 pairs)
    for ppm in (50000, 0):
        g.set_option("screen_floor_ppm", ppm)
        g.profile_reset()
        for j in range(6):  # one batch per call: each call's report is read by the next
            q = Q[32 * j:32 * (j + 1)]
            assert_same(*search_all(g, q, 2, 10, 32), *o.search(q, 2, 10))
        p = g.profile_read()
        if ppm:
            # calls 0, 4 screened (each trips: 3, then 6 exact batches), calls 1-3 and 5 exact
            assert p["screen_floor_trips"] == 2 and p["screen_floor_batches"] == 4, p
        else:
            assert p["screen_floor_trips"] == 0 and p["screen_floor_batches"] == 0, p


def test_screen_ties_duplicates_nonfinite_huge_subnormal():
    rng = np.random.default_rng(17)
    dim = 32
    base = rng.standard_normal((3000, dim)).astype(np.float32)
    X = np.concatenate([base, base, base[:500]])           # exact duplicate vectors: equal distances
    ids = np.concatenate([np.arange(3000), np.arange(3000) + 10000, np.arange(500)]).astype(np.uint64)
    # (no NaN: the reference ranks with std::partial_sort on (dist, id) pairs, and a NaN
    # key breaks its strict weak order, so where it lands is undefined behaviour)
    X[17, 3] = np.inf
    X[31, :] = -np.inf
    X[40, 5] = 3.0e38                                      # finite, overflows when squared
    X[41, 7] = 2.0e15                                      # above the screen's 2^50 limit
    X[42, :] = 1.0e-39                                     # subnormal coordinates (flushed in the shadow)
    X[43, 0] = 1.0e-40
    X[44, :8] = 1.5e-38
    lists = np.zeros(len(X), np.int64)
    lists[rng.random(len(X)) < 0.1] = 1
    C = np.zeros((2, dim), np.float32)
    C[1] = 5.0
    g, o = lists_pair(X, ids, lists, C, 0)
    Q = np.concatenate([base[:48] + 1e-3 * rng.standard_normal((48, dim)).astype(np.float32),
                        rng.standard_normal((40, dim)).astype(np.float32),
                        np.full((1, dim), 1e-39, np.float32),         # a subnormal query
                        np.zeros((1, dim), np.float32)])               # the zero query
    Q[60, 2] = 1.0e20                                                  # a huge query coordinate
    for k in (5, 10, 40):
        Dr, Ir = o.search(Q, 2, k)
        for defer in (1, 0):
            g.set_option("screen_defer", defer)
            assert_same(*search_all(g, Q, 2, k, 90), Dr, Ir)
            assert_same(*search_all(g, Q, 2, k, 7), Dr, Ir)


@pytest.mark.parametrize("dim", [1, 3, 67, 130, 256])
@pytest.mark.parametrize("metric", [0, 1])
def test_screen_odd_dimensions(dim, metric):
    X, ids, lists, C, Q = hub_data(dim, seed=dim + 7, n_hub=12000, n_other=800)
    g, o = lists_pair(X, ids, lists, C, metric)
    nprobe = 3 if metric == 0 else 6
    Dr, Ir = o.search(Q, nprobe, 10)
    for defer in (1, 0):
        g.set_option("screen_defer", defer)
        assert_same(*search_all(g, Q, nprobe, 10, 130), Dr, Ir)


def test_screen_rebuilt_after_incremental_adds_and_under_the_cap():
    X, Q, ids = oracle.reference_test_data(20000, 120, 64)
    nlist, nprobe, k = 32, 8, 10
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, nlist, vdb.Metric.L2, device=0))
    o = oracle.OracleIndex(64, nlist, 0)
    g.train(X[:5000])
    o.train(X[:5000])
    for a, b in ((0, 7000), (7000, 7001), (7001, 20000)):
        g.add(X[a:b], ids[a:b])
        o.add(X[a:b], ids[a:b])
        D, I, p = screen_stats(g, Q, nprobe, k, 64)
        assert_same(D, I, *o.search(Q, nprobe, k))
        assert p["bounded_blocks"] > 0, p
    # a residency cap that holds the lists: it counts list bytes only (the reference's
    # gpu_memory_used_), so the screen stays; a cap below them moves the lists to the tier
    # (the screen serves there with its shadow resident and the rows at home), lifting it
    # brings them back
    g.set_option("max_gpu_memory", int(20000 * (64 * 4 + 8) * 1.2))
    D, I, p = screen_stats(g, Q, nprobe, k, 64)
    assert_same(D, I, *o.search(Q, nprobe, k))
    assert p["bounded_blocks"] > 0, p
    g.set_option("max_gpu_memory", int(20000 * (64 * 4 + 8) * 0.6))
    D, I, p = screen_stats(g, Q, nprobe, k, 64)
    assert_same(D, I, *o.search(Q, nprobe, k))
    st = g.cache_stats()
    assert p["bounded_blocks"] > 0 and st["capacity_bytes"] > 0 and st["screen_resident"] == 1, (p, st)
    g.set_option("max_gpu_memory", 0)
    assert g.cache_stats()["capacity_bytes"] == 0
    D, I, p = screen_stats(g, Q, nprobe, k, 64)
    assert_same(D, I, *o.search(Q, nprobe, k))
    assert p["bounded_blocks"] > 0, p


@pytest.mark.parametrize("metric", [0, 1])
def test_screen_equals_exact_scan_on_trained_index(metric):
    """gpu_vs_cpu_test's shape with stale slots: screened and exact scans, and the oracle."""
    X, Q, ids = oracle.reference_test_data(30000, 300, 96)
    nlist = 64
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(96, nlist, vdb.Metric(metric), device=0))
    o = oracle.OracleIndex(96, nlist, metric)
    g.train(X[:8000])
    o.train(X[:8000])
    g.add(X, ids)
    o.add(X, ids)
    for nprobe, k in ((1, 10), (8, 10), (16, 64), (64, 3)):
        Dr, Ir = o.search(Q, nprobe, k)
        g.set_option("screen", 1)
        for defer in (0, 1):
            g.set_option("screen_defer", defer)
            assert_same(*search_all(g, Q, nprobe, k, 100), Dr, Ir)
        g.set_option("screen", 0)
        assert_same(*search_all(g, Q, nprobe, k, 100), Dr, Ir)


def test_footprint_is_the_device_memory_and_one_fp32_copy():
    """vdb_ivf_gpu_bytes_allocated is what the handle really holds (hipMemGetInfo deltas),
    and while the screen serves, the lists are held once in fp32 (the row-major copy) plus
    the bf16 shadow: ~1.5x the list bytes. Exact-path searches (k > 64, up to the server's
    1000) scan that row-major copy: no second fp32 copy, no arena rebuild (which would stall
    every batch in flight), results bit-identical."""
    import torch
    torch.cuda.set_device(0)
    dim, n = 256, 200000
    X, Q, ids = oracle.reference_test_data(n, 64, dim)

    def build():
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, 64, vdb.Metric.L2, device=0))
        g.train(X[:20000])
        g.add(X, ids)
        g.search(Q, nprobe=8, k=10)  # (builds the screen)
        return g

    del_g = build()  # (every kernel and runtime object loaded once)
    for k in (65, 100, 1000):  # (and the exact kernels' scratch memory, which the runtime keeps)
        del_g.search(Q[:4], nprobe=8, k=k)
    del del_g
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    g = build()
    free1 = torch.cuda.mem_get_info(0)[0]
    alloc = g.gpu_bytes_allocated()
    used = free0 - free1
    lists = n * dim * 4
    print("footprint", alloc, "device delta", used, "list bytes", lists)
    assert abs(used - alloc) <= 0.03 * alloc + (48 << 20), (used, alloc)
    assert alloc <= 1.6 * lists + (64 << 20), (alloc, lists)
    o = oracle.OracleIndex(dim, 64, 0)
    o.centroids = g.centroids
    o.add(X, ids)
    for k in (65, 100, 1000):  # exact path over the row-major copy
        assert_same(*g.search(Q, nprobe=8, k=k), *o.search(Q, 8, k))
        alloc2 = g.gpu_bytes_allocated()
        # (the workspaces grow with k: partials of k entries per segment)
        assert alloc2 <= 1.6 * lists + (256 << 20), (k, alloc, alloc2)
        free2 = torch.cuda.mem_get_info(0)[0]
        assert abs((free0 - free2) - alloc2) <= 0.03 * alloc2 + (48 << 20), (free0 - free2, alloc2)
    assert_same(*g.search(Q, nprobe=8, k=10), *o.search(Q, 8, 10))  # (and the screen again)
    # the screen off: the interleaved arena comes back in place of the rows and the shadow
    g.set_option("screen", 0)
    assert g.gpu_bytes_allocated() <= 1.15 * lists + (256 << 20), g.gpu_bytes_allocated()
    assert_same(*g.search(Q, nprobe=8, k=65), *o.search(Q, 8, 65))


@pytest.mark.parametrize("metric", [0, 1])
def test_automatic_shadow_at_large_nprobe(metric):
    """The automatic shadow format (screen_i8 = 2) is calibrated by one screened batch of the
    index's own vectors at the nprobe of the search that builds the screen. At nprobe 300 a
    64-query batch holds 19,200 (query, probe) pairs, above the plan kernel's 8,192: the
    calibration batch is cut like every batch (batch_cap); before that fix this search faulted
    on the GPU. Results stay exact, the format built is reported, and 32-query items (nprobe
    >= 64) serve k = 64."""
    from test_gpu_parity import mirror_from_oracle
    rng = np.random.default_rng(700 + metric)
    dim, nlist, nprobe = 96, 300, 300
    X = rng.standard_normal((20000, dim)).astype(np.float32)
    Q = rng.standard_normal((70, dim)).astype(np.float32)
    ids = np.arange(len(X), dtype=np.uint64)
    o = oracle.OracleIndex(dim, nlist, metric)
    o.centroids = X[:nlist] * 0.3
    o.add(X, ids)
    for k in (10, 64):
        g = mirror_from_oracle(o, dim, nlist, metric)
        g.add(X, ids)
        # (the first search builds and calibrates the screen; the statistics below are then
        # this k's own batches: the calibration batch never counts into them)
        assert_same(*g.search(Q[:8], nprobe=nprobe, k=k), *o.search(Q[:8], nprobe, k))
        D, I, p = screen_stats(g, Q, nprobe, k, 70)
        assert_same(D, I, *o.search(Q, nprobe, k))
        assert p["screen_shadow"] in (1, 2), p
        assert p["bounded_blocks"] > 0, p  # (the screen served it)
    # the search that builds (and calibrates) the screen reports its own batches only: the
    # blocks it screened equal those of the same search on the built screen
    g = mirror_from_oracle(o, dim, nlist, metric)
    g.add(X, ids)
    _, _, p1 = screen_stats(g, Q, nprobe, 10, 70)
    _, _, p2 = screen_stats(g, Q, nprobe, 10, 70)
    assert p1["bounded_blocks"] == p2["bounded_blocks"] > 0, (p1, p2)
