"""CPU tests of the oracle (oracle/cpu_ref.cpp), the restatement of the reference's
IVF-Flat CPU path (engine/ivf_flat_index.cpp, use_gpu=false).

The reference's own tests pin no values, so the oracle is pinned by:
the known answer the reference benchmark implies (query i == vector i,
bench/benchmark.cpp:130-138), its validity rules (gpu_vs_cpu_test.cpp:209-219,
simple_test.cpp:186), an independent numpy restatement (oracle/np_ref.py), brute-force
equivalence at nprobe == nlist, and the committed golden fixtures (tests/golden).
"""
import glob
import os

import numpy as np
import pytest

import oracle
import oracle.np_ref as npr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
U64MAX = np.iinfo(np.uint64).max


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def lists_of(o):
    return [o.get_list(l) for l in range(o.nlist)]


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("nprobe,k", [(1, 1), (3, 7), (8, 20)])
def test_oracle_equals_numpy_restatement(metric, nprobe, k):
    X, Q, ids = oracle.reference_test_data(1500, 25, 24, seed=100 + metric)
    o = oracle.OracleIndex(24, 8, metric)
    o.train(X[:400])
    o.add(X, ids)
    D, I = o.search(Q, nprobe, k)
    Dn, In = npr.search(metric, o.centroids, lists_of(o), Q, nprobe, k)
    assert np.array_equal(I, In)
    assert np.array_equal(bits(D), bits(Dn))
    for q in Q[:5]:
        assert np.array_equal(o.select_nprobe(q, nprobe), npr.select_nprobe(metric, o.centroids, q, nprobe))
    assert np.array_equal(o.assign(X[:300]), npr.assign(metric, o.centroids, X[:300]))


def test_lloyd_from_kmeanspp_seeds():
    X, _, _ = oracle.reference_test_data(2000, 1, 16, seed=9)
    full = oracle.OracleIndex(16, 10, 0)
    full.train(X)
    seeds = oracle.OracleIndex(16, 10, 0)
    seeds.train_seed_only(X)
    # every k-means++ seed is one of the training vectors (ivf_flat_index.cpp:57-101)
    C0 = seeds.centroids
    assert all(np.any(np.all(X == c, axis=1)) for c in C0)
    assert np.array_equal(bits(npr.lloyd(0, X, C0)), bits(full.centroids))


def test_benchmark_kat_self_query():
    """bench/benchmark.cpp re-seeds mt19937(42) for queries: query i is vector i, so
    its top-1 is (i, 0.0f) — add and select_nprobe compute the same argmin."""
    X = oracle.gen_normal(42, 1000 * 64).reshape(1000, 64)
    Q = oracle.gen_normal(42, 200 * 64).reshape(200, 64)
    assert np.array_equal(Q, X[:200])
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, np.arange(1000, dtype=np.uint64))
    D, I = o.search(Q, 5, 10)
    assert np.array_equal(I[:, 0], np.arange(200, dtype=np.uint64))
    assert np.all(bits(D[:, 0]) == 0)


def test_validity_rules():
    """gpu_vs_cpu_test.cpp:209-219 and simple_test.cpp:186."""
    X, Q, ids = oracle.reference_test_data(10000, 100, 64)
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, ids)
    D, I = o.search(Q, 8, 10)
    assert np.all((I < 10000) | (I == U64MAX))
    assert np.all(np.isfinite(D)) and np.all(D >= 0)
    assert np.all(np.diff(D, axis=1) >= 0)
    assert o.total_vectors == 10000


def test_nprobe_equals_nlist_is_bruteforce():
    X, Q, ids = oracle.reference_test_data(2000, 15, 12, seed=4)
    o = oracle.OracleIndex(12, 20, 0)
    o.centroids = X[:20]
    o.add(X, ids)
    D, I = o.search(Q, 20, 10)
    full = npr.distances(0, Q, X)
    for q in range(len(Q)):
        order = np.lexsort((ids, full[q]))[:10]
        assert np.array_equal(I[q], ids[order])
        assert np.array_equal(bits(D[q]), bits(full[q][order]))


def test_stale_slot_quirk_is_reproduced():
    """ivf_flat_index.cpp:210-233: an empty probed list keeps the previous query's slot."""
    rng = np.random.default_rng(3)
    X = rng.standard_normal((600, 6)).astype(np.float32)
    C = np.concatenate([X[:4], np.full((4, 6), 50.0, np.float32)])
    o = oracle.OracleIndex(6, 8, 0)
    o.centroids = C
    o.add(X, np.arange(600, dtype=np.uint64))
    assert sum(o.list_count(l) == 0 for l in range(8)) == 4
    Q = rng.standard_normal((12, 6)).astype(np.float32) * 8
    D, I = o.search(Q, 6, 5)
    Dn, In = npr.search(0, C, lists_of(o), Q, 6, 5)
    assert np.array_equal(I, In) and np.array_equal(bits(D), bits(Dn))
    # one query per call: no earlier query, so no leaked slots — results can differ
    D1 = np.concatenate([o.search(q[None], 6, 5)[0] for q in Q])
    assert np.array_equal(bits(D1[0]), bits(D[0]))


def test_multithreaded_search_equals_serial():
    X, Q, ids = oracle.reference_test_data(5000, 64, 32, seed=12)
    o = oracle.OracleIndex(32, 16, 0)
    o.train(X[:2000])
    o.add(X, ids)
    D1, I1 = o.search(Q, 4, 10, threads=1)
    D2, I2 = o.search(Q, 4, 10, threads=4)
    assert np.array_equal(I1, I2) and np.array_equal(bits(D1), bits(D2))


@pytest.mark.parametrize("metric", [0, 1])
def test_multithreaded_assign_equals_serial(metric):
    # the OpenMP assignment the full-scale GPU assignment tests check against: every row's
    # argmin identical to the serial assign_to_lists (cpp:259-295) and to the numpy one,
    # including ties (duplicated centroids go to the lowest index)
    rng = np.random.default_rng(40 + metric)
    X = rng.standard_normal((3000, 48)).astype(np.float32)
    C = rng.standard_normal((100, 48)).astype(np.float32)
    C[7] = C[3]
    X[:50] = C[3]
    o = oracle.OracleIndex(48, 100, metric)
    o.centroids = C
    a1 = o.assign(X)
    for t in (0, 3, 8):
        assert np.array_equal(o.assign(X, threads=t), a1)
    assert np.array_equal(a1, npr.assign(metric, C, X))
    if metric == 0:
        assert np.all(a1[:50] == 3)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_decomposition(world):
    """Per-rank partials over the lists each rank owns, merged, equal the full search
    (the protocol of the list-sharded multi-GPU path)."""
    X, Q, ids = oracle.reference_test_data(6000, 40, 16, seed=world)
    o = oracle.OracleIndex(16, 24, 0)
    o.train(X[:3000])
    o.add(X, ids)
    D, I = o.search(Q, 7, 10)
    rng = np.random.default_rng(world)
    owner = rng.integers(0, world, 24)
    parts = [o.search_shard(Q, 7, 10, (owner == r).astype(np.uint8)) for r in range(world)]
    Dm, Im = oracle.merge_ranks(np.stack([p[0] for p in parts]), np.stack([p[1] for p in parts]), 10)
    assert np.array_equal(Im, I) and np.array_equal(bits(Dm), bits(D))
    for r in range(world):  # the parallel shard search (large-config GPU tests) is bit-identical
        Dt, It = o.search_shard(Q, 7, 10, (owner == r).astype(np.uint8), threads=4)
        assert np.array_equal(It, parts[r][1]) and np.array_equal(bits(Dt), bits(parts[r][0]))


def test_count_only_lists_keep_shard_results():
    """bench.py --shard-check: lists of other shards kept as counts only (no rows) give the
    same shard partials as fully stored lists, empty lists (stale slots) included."""
    X, Q, ids = oracle.reference_test_data(3000, 30, 16, seed=9)
    o = oracle.OracleIndex(16, 40, 0)
    o.centroids = np.concatenate([X[:32], np.full((8, 16), 50.0, np.float32)])  # 8 empty lists
    o.add(X, ids)
    owned = (np.arange(40) % 3 == 0).astype(np.uint8)
    D, I = o.search_shard(Q, 36, 10, owned)
    c = oracle.OracleIndex(16, 40, 0)
    c.centroids = o.centroids
    for l in range(40):
        v, i = o.get_list(l)
        if owned[l]:
            bv, bi = c.list_buffers(l, len(i))
            bv[...] = v
            bi[...] = i
        else:
            c.set_list_count(l, len(i))
    Dc, Ic = c.search_shard(Q, 36, 10, owned)
    assert np.array_equal(Ic, I) and np.array_equal(bits(Dc), bits(D))
    # streamed: one owned probed list holds rows at a time (bench.py's full-shard check)
    s = oracle.OracleIndex(16, 40, 0)
    s.centroids = o.centroids
    counts = [o.list_count(l) for l in range(40)]
    filled = []

    def fill(l, v, i):
        filled.append(l)
        v[...], i[...] = o.get_list(l)

    Ds, Is, loaded = s.search_shard_streamed(Q, 36, 10, owned, counts, fill, threads=3)
    assert np.array_equal(Is, I) and np.array_equal(bits(Ds), bits(D))
    assert len(set(filled)) == len(filled) and all(owned[l] for l in filled)
    assert loaded == sum(counts[l] for l in filled) > 0


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_golden_fixture(path):
    f = np.load(path)
    dim, nlist, train_n, nprobe, k, metric = (int(x) for x in f["params"])
    o = oracle.OracleIndex(dim, nlist, metric)
    if train_n:
        o.train(f["X"][:train_n])
        assert np.array_equal(bits(o.centroids), bits(f["centroids"]))
    else:
        o.centroids = f["centroids"]
    o.add(f["X"], f["ids"])
    assert np.array_equal(np.array([o.list_count(l) for l in range(nlist)], np.uint64), f["list_sizes"])
    D, I = o.search(f["Q"], nprobe, k)
    assert np.array_equal(I, f["I"]) and np.array_equal(bits(D), bits(f["D"]))
