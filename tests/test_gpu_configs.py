"""GPU parity at the BASELINE.json configurations' own sizes (configs[0] and configs[1]);
configs[2] (10M x 768, the bench) is checked inside bench.py on a query sample
(`cpu_baseline.parity_with_gpu`), and the 8-GPU configs through the sharding tests.

* cfg1 — 100K x 128, gpu_vs_cpu_test.cpp's generator (mt19937(12345), database then queries):
  brute force (nlist 1) and the test's own IVF setup (nlist 128, nprobe 8, train on 10 000,
  gpu_vs_cpu_test.cpp:24-32, 147), train included: centroids, list membership and results
  must equal the oracle's bit for bit.
* cfg2 — 1M x 768, nlist 256, nprobe 16, batch 64: the bench's build (device-generated data,
  train on 100K, add 1M); the oracle gets the GPU's centroids and the probed lists, and one
  batch of 64 queries must match ids and distance bits.
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb

vdb = load_vdb()
pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_cfg1_bruteforce_100k_x_128():
    X, Q, ids = oracle.reference_test_data(100_000, 1000, 128)
    o = oracle.OracleIndex(128, 1, 0)
    o.centroids = np.zeros((1, 128), np.float32)
    o.add(X, ids)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(128, 1))
    g.centroids = np.zeros((1, 128), np.float32)
    g.add(X, ids)
    D, I = g.search(Q, nprobe=1, k=10)
    Dr, Ir = o.search(Q, 1, 10, threads=16)
    assert np.array_equal(I, Ir)
    assert np.array_equal(bits(D), bits(Dr))
    assert np.all(np.isfinite(D)) and np.all(D >= 0) and np.all(I < 100_000)   # gpu_vs_cpu_test.cpp:209-219


def test_cfg1_ivf_train_and_search_100k_x_128():
    X, Q, ids = oracle.reference_test_data(100_000, 1000, 128)
    o = oracle.OracleIndex(128, 128, 0)
    o.train(X[:10_000])
    o.add(X, ids)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(128, 128))
    g.train(X[:10_000])
    assert np.array_equal(bits(g.centroids), bits(o.centroids)), "train() differs from the reference algorithm"
    g.add(X, ids)
    assert np.array_equal(g.list_sizes(), np.array([o.list_count(l) for l in range(128)], np.uint64))
    D, I = g.search(Q, nprobe=8, k=10)
    Dr, Ir = o.search(Q, 8, 10, threads=16)
    assert np.array_equal(I, Ir)
    assert np.array_equal(bits(D), bits(Dr))


@pytest.mark.parametrize("data", ["iid", "mixture"])
def test_cfg2_1m_x_768_nlist256_nprobe16_batch64(data):
    """`mixture`: bench.py --data mixture's generator (256 Gaussian components in super-clusters
    of 16), balanced lists probed by few queries each — the narrow-item regime of clustered data."""
    import torch
    n, dim, nlist, nprobe, B, k = 1_000_000, 768, 256, 16, 64, 10
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        s = torch.cuda.current_stream().cuda_stream
        data_t = torch.empty((n, dim), dtype=torch.float32, device=dev)
        q = torch.empty((B, dim), dtype=torch.float32, device=dev)
        if data == "mixture":  # bench.py's two-level mixture: super-clusters of nprobe components
            import bench
            centers = bench.mixture_centers(vdb, nlist, nprobe, dim, 0.35, dev)
            vdb.gen_mixture_device(data_t.data_ptr(), n, dim, centers.data_ptr(), nlist, 0.1, 12345, 0, s)
            vdb.gen_mixture_device(q.data_ptr(), B, dim, centers.data_ptr(), nlist, 0.1, 12346, 0, s)
        else:
            vdb.gen_normal_device(data_t.data_ptr(), n * dim, seed=12345, stream=s)
            vdb.gen_normal_device(q.data_ptr(), B * dim, seed=12346, stream=s)
        ids = torch.arange(n, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist))
        g.train_device(data_t.data_ptr(), 100_000)
        g.add_device(data_t.data_ptr(), ids.data_ptr(), n)
        od = torch.empty((B, k), dtype=torch.float32, device=dev)
        oi = torch.empty((B, k), dtype=torch.int64, device=dev)
        g.search_device(q.data_ptr(), B, nprobe, k, od.data_ptr(), oi.data_ptr(), s)
        torch.cuda.synchronize()
        Q = q.cpu().numpy()
        D, I = od.cpu().numpy(), oi.cpu().numpy().view(np.uint64)
        if data == "mixture":  # the generator: chunked calls give the same rows
            part = torch.empty((1000, dim), dtype=torch.float32, device=dev)
            vdb.gen_mixture_device(part.data_ptr(), 1000, dim, centers.data_ptr(), nlist, 0.1, 12345, 5000, s)
            torch.cuda.synchronize()
            assert torch.equal(part, data_t[5000:6000])
        del data_t, ids
    o = oracle.OracleIndex(dim, nlist, 0)
    o.centroids = g.centroids
    sizes = g.list_sizes()
    assert int(sizes.sum()) == n
    if data == "mixture":  # mostly one component per list (k-means merges a few), no hub lists
        assert np.median(sizes) > 0.75 * n / nlist and sizes.max() < 8 * n / nlist
    probed = sorted({int(l) for qv in Q for l in o.select_nprobe(qv, nprobe)})
    for l in probed:  # only the probed lists are ever read for these queries
        v, i = o.list_buffers(l, int(sizes[l]))
        if len(i):
            g.get_list_into(l, v, i)
    Dr, Ir = o.search(Q, nprobe, k, threads=16)
    assert np.array_equal(I, Ir)
    assert np.array_equal(bits(D), bits(Dr))
