"""GPU: the list-cache tier (option list_cache_bytes), the reference's residency model
(load_list_to_gpu on first touch under a byte cap, evict_list_from_gpu, warmup_lists,
get_gpu_memory_usage: ivf_flat_index.cpp:387-471, 690-709). Lists live in page-locked
host memory and HBM caches whole lists; results must stay bit-identical to the oracle
whatever the cache holds: with evictions, batches split because their probed lists
overflow the cache, fragmented caches repacked, empty lists (stale slots), the tier
switched on before or after add, and switched off again. These cases exercise the
list-cache path itself, so the screen is off here (option "screen" 0): with it, L2 / IP
searches with k <= 64 keep the lists' shadow in HBM and never load lists into the cache
(the screened tier: test_gpu_screen_tier.py)."""
import numpy as np
import pytest

import oracle
from conftest import load_vdb
from test_gpu_parity import assert_same, bits

vdb = load_vdb()
pytestmark = pytest.mark.gpu

D, NLIST, NPROBE, K = 64, 64, 8, 10
BLOCK_BYTES = 64 * (D * 4 + 8)  # one 64-vector block of the arena (dp = 64 here)


def fixture():
    X, Q, ids = oracle.reference_test_data(20000, 300, D, seed=5)
    o = oracle.OracleIndex(D, NLIST, 0)
    o.train(X[:5000])
    o.add(X, ids)
    blocks = np.array([(o.list_count(l) + 63) // 64 for l in range(NLIST)])
    need = max(int(blocks[o.select_nprobe(q, NPROBE)].sum()) for q in Q)  # one query's probed lists
    return X, Q, ids, o, blocks, need


def make(o, X, ids, cache_bytes, before_add):
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST))
    g.set_option("screen", 0)
    g.centroids = o.centroids
    if before_add:
        g.set_option("list_cache_bytes", cache_bytes)
        g.add(X, ids)
    else:
        g.add(X, ids)
        g.set_option("list_cache_bytes", cache_bytes)
    return g


@pytest.mark.parametrize("before_add", [True, False])
def test_cache_tier_matches_oracle_under_eviction(before_add):
    X, Q, ids, o, blocks, need = fixture()
    cap = (need + 8) * BLOCK_BYTES          # barely more than one query's lists
    g = make(o, X, ids, cap, before_add)
    Dr, Ir = o.search(Q, NPROBE, K)
    for batch in (256, 16, 1):              # 256 and 16 overflow the cache and are split
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    st = g.cache_stats()
    assert st["capacity_bytes"] == (cap // BLOCK_BYTES) * BLOCK_BYTES
    assert st["loads"] > NLIST and st["evictions"] > 0
    assert 0 < st["resident_bytes"] <= st["capacity_bytes"]
    assert 0 < g.get_gpu_memory_usage() <= st["resident_bytes"]   # count * (D * 4 + 8) per cached list
    assert g.gpu_bytes_allocated() >= st["capacity_bytes"]
    for l in (0, 17, NLIST - 1):            # host-resident arena still exports lists
        assert np.array_equal(g.get_list(l)[1], o.get_list(l)[1])


def test_cache_tier_large_cache_hits_and_off_again():
    X, Q, ids, o, blocks, need = fixture()
    g = make(o, X, ids, int(blocks.sum() + 1) * BLOCK_BYTES, True)   # everything fits
    Dr, Ir = o.search(Q, NPROBE, K)
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    loads = g.cache_stats()["loads"]
    assert loads <= NLIST
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)  # second pass: all hits
    st = g.cache_stats()
    assert st["loads"] == loads and st["evictions"] == 0
    g.set_option("list_cache_bytes", 0)                      # arena back in HBM
    assert g.cache_stats()["capacity_bytes"] == 0
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)


def test_warmup_evict_and_too_small_cache():
    X, Q, ids, o, blocks, need = fixture()
    big = int(np.argmax(blocks))
    cap = (int(blocks.max()) + 2) * BLOCK_BYTES
    g = make(o, X, ids, cap, True)
    g.warmup_lists([big])
    st = g.cache_stats()
    assert st["resident_lists"] == 1 and st["resident_bytes"] == int(blocks[big]) * BLOCK_BYTES
    small = [l for l in np.argsort(blocks)[:3].tolist() if blocks[l] > 0]
    g.warmup_lists(small)                   # LRU: the big list makes room when needed
    st = g.cache_stats()
    assert st["resident_lists"] >= len(small)
    g.evict_list(small[0])
    assert g.cache_stats()["resident_lists"] == st["resident_lists"] - 1
    g.evict_list(small[0])                  # evicting a non-resident list is a no-op
    if need > cap // BLOCK_BYTES:
        with pytest.raises(vdb.VdbError, match="list_cache_bytes"):
            g.search(Q, nprobe=NPROBE, k=K)
    with pytest.raises(vdb.VdbError):
        g.set_option("list_cache_bytes", BLOCK_BYTES - 1)   # below one block


def test_cache_tier_empty_lists_stale_slots():
    """Quirk A1 (empty probed lists keep the previous query's slot) across split batches."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3000, 16)).astype(np.float32)
    Q = rng.standard_normal((300, 16)).astype(np.float32)
    ids = np.arange(3000, dtype=np.uint64)
    C = np.concatenate([X[:10], 6.0 + rng.standard_normal((6, 16)).astype(np.float32) * 0.1])
    C[10:] *= np.where(rng.random((6, 1)) < 0.5, -1, 1).astype(np.float32)
    o = oracle.OracleIndex(16, 16, 0)
    o.centroids = C
    o.add(X, ids)
    assert any(o.list_count(l) == 0 for l in range(16))
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(16, 16))
    g.centroids = C
    g.add(X, ids)
    dp = 64                                  # 16 dims pad to one 64-float row
    blocks = sorted(((o.list_count(l) + 63) // 64 for l in range(16)), reverse=True)
    g.set_option("list_cache_bytes", (sum(blocks[:12]) + 1) * 64 * (dp * 4 + 8))
    Dr, Ir = o.search(Q, 12, 8)
    for batch in (256, 7):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=12, k=8), Dr, Ir)
    assert np.all(bits(Dr) == bits(g.search(Q, nprobe=12, k=8)[0]))


@pytest.mark.parametrize("dim", [64, 70])
def test_lists_served_from_file(tmp_path, dim):
    """The tier's home on disk (vdb_ivf_open_lists): a saved index is served without
    loading its lists; they are read, padded and interleaved on demand. Results,
    get_list and the read-only contract must hold; dim 70 exercises row padding."""
    X, Q, ids = oracle.reference_test_data(20000, 200, dim, seed=9)
    o = oracle.OracleIndex(dim, NLIST, 0)
    o.train(X[:5000])
    o.add(X, ids)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "index.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    h.set_option("screen", 0)
    dp = 128 if dim > 64 else 64
    blocks = np.array([(o.list_count(l) + 63) // 64 for l in range(NLIST)])
    need = max(int(blocks[o.select_nprobe(q, NPROBE)].sum()) for q in Q)
    h.set_option("list_cache_bytes", (need + 8) * 64 * (dp * 4 + 8))
    h.open_lists(path)
    assert h.get_total_vectors() == len(X)
    assert np.array_equal(bits(h.centroids), bits(o.centroids))
    Dr, Ir = o.search(Q, NPROBE, K)
    for batch in (256, 1):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    st = h.cache_stats()
    assert st["loads"] > 0 and st["evictions"] > 0 and st["file_bytes_read"] > 0
    for l in (0, 31, NLIST - 1):
        v, i = h.get_list(l)
        ov, oi = o.get_list(l)
        assert np.array_equal(i, oi) and np.array_equal(bits(v), bits(ov))
    with pytest.raises(vdb.VdbError, match="read-only"):
        h.add(X[:10], ids[:10])
    h.warmup_lists(list(range(NLIST)))       # LRU keeps what fits; results unchanged
    assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)


def test_tier_pipeline_file_home_next_use_and_prefetch(tmp_path):
    """A call of many queries against a file home with a cache that holds a few queries'
    lists: the call is cut into sub-batches that fit, each next sub-batch's lists are read
    (io_uring, O_DIRECT where allowed) while the current one scans, and evictions follow
    the call's known next uses. Results bit-identical to the oracle, stale slots included."""
    X, Q, ids, o, blocks, need = fixture()
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "tier.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST))
    h.set_option("screen", 0)
    h.set_option("list_cache_bytes", (3 * need + 8) * BLOCK_BYTES)   # room for ~3 queries' lists at once
    h.open_lists(path)
    Dr, Ir = o.search(Q, NPROBE, K)
    for batch in (64, 5):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    st = h.cache_stats()
    assert st["subbatches"] > 2 * len(Q) // 64 and st["prefetches"] > 0, st
    assert st["file_bytes_read"] > 0 and st["loads"] > 0
    assert st["io_uring"] in (0, 1) and st["o_direct"] in (0, 1)
    # a second pass over the same calls: next-use eviction never needs more reads than
    # one full load of every list per sub-batch
    before = st["file_bytes_read"]
    h.set_batch(64)
    assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    assert h.cache_stats()["file_bytes_read"] - before <= int(blocks.sum()) * 64 * (D * 4 + 8) * len(Q)


def test_tier_concurrent_streams_under_eviction():
    """Three searches in flight on three streams while the cache evicts and reloads
    (host-memory home): every stream's results equal the oracle's (a search on
    another stream must wait for lists and directory entries still being copied)."""
    import torch
    X, Q, ids, o, blocks, need = fixture()
    g = make(o, X, ids, (2 * need + 8) * BLOCK_BYTES, False)
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(Q).to(dev)
    n = len(Q) // 3
    od = torch.empty((3 * n, K), dtype=torch.float32, device=dev)
    oi = torch.empty((3 * n, K), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    for rep in range(3):
        for j, s in enumerate(streams):
            g.search_device(q[j * n:].data_ptr(), n, NPROBE, K, od[j * n:].data_ptr(), oi[j * n:].data_ptr(),
                            s.cuda_stream)
        torch.cuda.synchronize()
        for j in range(3):
            assert_same(od[j * n:(j + 1) * n].cpu().numpy(), oi[j * n:(j + 1) * n].cpu().numpy().view(np.uint64),
                        *o.search(Q[j * n:(j + 1) * n], NPROBE, K))
    assert g.cache_stats()["evictions"] > 0
