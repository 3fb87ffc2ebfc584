"""Generate the committed golden fixtures (tests/golden/*.npz) from the oracle.

Each fixture holds the inputs the reference's own tests use (or a hand-built edge
case) and the expected outputs of the reference CPU path restatement
(oracle/cpu_ref.cpp): trained centroids, list sizes, and (ids, distance bits) of the
search. Inputs that come from std::mt19937 + std::normal_distribution<float> are
stored too, so a fixture is self-contained data.

Run: python tests/golden/make_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402


def save(name, **arrays):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    print("wrote", name, {k: v.shape for k, v in arrays.items()})


def trained_case(name, X, Q, ids, dim, nlist, train_n, nprobe, k, metric=0):
    o = oracle.OracleIndex(dim, nlist, metric)
    o.train(X[:train_n])
    o.add(X, ids)
    D, I = o.search(Q, nprobe, k)
    save(name, X=X, Q=Q, ids=ids, params=np.array([dim, nlist, train_n, nprobe, k, metric], np.int64),
         centroids=o.centroids, list_sizes=np.array([o.list_count(l) for l in range(nlist)], np.uint64),
         D=D, I=I)


def main():
    # test/simple_test.cpp:111-165 — mt19937(42): database then queries.
    flat = oracle.gen_normal(42, (1000 + 10) * 64)
    trained_case("simple_test", flat[:64000].reshape(1000, 64), flat[64000:].reshape(10, 64),
                 np.arange(1000, dtype=np.uint64), 64, 16, 100, 4, 5)
    # test/CMakeLists.txt:56 — gpu_vs_cpu_test 10000 100 64 32 (nprobe 8, k 10, train 10000).
    X, Q, ids = oracle.reference_test_data(10000, 100, 64)
    trained_case("gpu_vs_cpu_ctest", X, Q, ids, 64, 32, 10000, 8, 10)
    # bench/CMakeLists.txt:48 — benchmark 1000 64 32 5 (k 10); the re-seeded generator makes
    # query i == vector i (benchmark.cpp:130-138), 64 of its 10000 queries kept.
    X = oracle.gen_normal(42, 1000 * 64).reshape(1000, 64)
    Q = oracle.gen_normal(42, 64 * 64).reshape(64, 64)
    trained_case("benchmark_small", X, Q, np.arange(1000, dtype=np.uint64), 64, 32, 1000, 5, 10)
    # Inner product, small.
    X, Q, ids = oracle.reference_test_data(3000, 20, 16, seed=3)
    trained_case("inner_product", X, Q, ids, 16, 12, 3000, 3, 7, metric=1)
    # Hand-built: empty lists (stale-slot reuse), duplicate vectors and ids.
    rng = np.random.default_rng(0)
    base = rng.standard_normal((400, 8)).astype(np.float32)
    X = np.concatenate([base, base[:50]])
    ids = np.concatenate([np.arange(400), np.arange(25), np.arange(900, 925)]).astype(np.uint64)
    C = np.concatenate([base[:6], np.full((4, 8), 40.0, np.float32) * np.arange(1, 5, dtype=np.float32)[:, None]])
    Q = np.concatenate([base[:10], rng.standard_normal((30, 8)).astype(np.float32)])
    o = oracle.OracleIndex(8, 10, 0)
    o.centroids = C
    o.add(X, ids)
    D, I = o.search(Q, 8, 6)
    save("empty_lists_dups", X=X, Q=Q, ids=ids, params=np.array([8, 10, 0, 8, 6, 0], np.int64), centroids=C,
         list_sizes=np.array([o.list_count(l) for l in range(10)], np.uint64), D=D, I=I)


if __name__ == "__main__":
    main()
