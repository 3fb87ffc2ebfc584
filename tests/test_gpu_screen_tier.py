"""GPU: the screened scan inside the list-cache tier (configs[4]'s shape: a shard larger than
HBM). The lists' bf16 shadow, norms and ids stay HBM-resident; the fp32 rows stay at the
home and only the exact re-checks' rows are read per batch: from page-locked host memory over
PCIe, or from the index file (io_uring, one read per survivor row). Exact-path searches
(k > 64) on the same handle go through the list cache, under eviction. Every result is
compared bit for bit with the oracle (ivf_flat_index.cpp:205-256 restated); the residency
model is the reference's load_list_to_gpu / evict_list_from_gpu (ivf_flat_index.cpp:387-471)
and its list streaming design (engine/prefetcher.h:139-183).
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb
from test_gpu_parity import assert_same

vdb = load_vdb()
pytestmark = pytest.mark.gpu

NLIST, NPROBE = 64, 8


def data(dim, metric=0, n=20000, nq=300, seed=5):
    X, Q, ids = oracle.reference_test_data(n, nq, dim, seed=seed)
    o = oracle.OracleIndex(dim, NLIST, metric)
    o.train(X[:5000])
    o.add(X, ids)
    return X, Q, ids, o


def block_bytes(dim):
    dp = -(-dim // 64) * 64
    return 64 * (dp * 4 + 8)


def need_blocks(o, Q, nprobe):
    blocks = np.array([(o.list_count(l) + 63) // 64 for l in range(NLIST)])
    return max(int(blocks[o.select_nprobe(q, nprobe)].sum()) for q in Q)


@pytest.mark.parametrize("metric", [0, 1])
def test_screened_tier_host_home_mixed_k(metric):
    """Lists homed in page-locked host memory (the tier entered by list_cache_bytes): k <= 64
    is served by the resident shadow with the survivors' rows read over PCIe, k > 64 by the
    list cache under eviction, interleaved on one handle."""
    dim = 64
    X, Q, ids, o = data(dim, metric)
    nprobe = NPROBE if metric == 0 else 2 * NPROBE
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST, vdb.Metric(metric), max_gpu_memory=0))
    g.centroids = o.centroids
    g.add(X, ids)
    g.set_option("list_cache_bytes", (need_blocks(o, Q, nprobe) + 8) * block_bytes(dim))
    for k in (10, 1, 64, 100, 10, 65, 16):
        Dr, Ir = o.search(Q, nprobe, k)
        for batch in (256, 17):
            g.set_batch(batch)
            assert_same(*g.search(Q, nprobe=nprobe, k=k), Dr, Ir)
    st = g.cache_stats()
    assert st["screen_resident"] == 1 and st["screen_batches"] > 0, st
    assert st["evictions"] > 0, st  # (the k > 64 searches)
    # shadow 2 dp + norms 16 + ids 8 bytes per vector (plus block padding): well below the lists
    assert st["screen_bytes"] < 0.7 * len(X) * (dim * 4 + 8), st


@pytest.mark.parametrize("rc", [0, 1], ids=["file_rows", "row_cache"])
@pytest.mark.parametrize("i8", [0, 1], ids=["bf16", "int8"])
@pytest.mark.parametrize("dim", [64, 70])
def test_screened_tier_file_home(tmp_path, dim, i8, rc):
    """Lists served from an index file: the shadow is built by streaming the file once;
    per batch only the survivors' rows are read (far fewer bytes than the probed lists),
    from the file, or (tier_row_cache) copied from the idle HBM cache filled with the
    largest lists. dim 70 pads the fetched rows to 128."""
    X, Q, ids, o = data(dim, seed=9)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "index.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    h.set_option("screen_i8", i8)
    h.set_option("tier_row_cache", rc)
    h.set_option("list_cache_bytes", (need_blocks(o, Q, NPROBE) + 8) * block_bytes(dim))
    h.open_lists(path)
    Dr, Ir = o.search(Q, NPROBE, 10)
    loads0 = None
    for batch in (256, 5):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=NPROBE, k=10), Dr, Ir)
        loads0 = h.cache_stats()["loads"] if loads0 is None else loads0
    st = h.cache_stats()
    assert st["screen_resident"] == 1 and st["loads"] == loads0, st  # (no per-batch loads)
    assert (st["loads"] > 0) == bool(rc) and (st["screen_rows_cached"] > 0) == bool(rc), st
    assert 0 < st["screen_rows_fetched"] and st["screen_row_bytes"] == st["screen_rows_fetched"] * dim * 4, st
    probed = sum(o.list_count(l) for q in Q for l in o.select_nprobe(q, NPROBE))
    rows = st["screen_rows_fetched"] + st["screen_rows_cached"]
    assert rows < (0.3 if i8 else 0.1) * probed * 2, st  # (two passes above)
    # k > 64 on the same handle: the list cache, under eviction
    Dr, Ir = o.search(Q, NPROBE, 80)
    assert_same(*h.search(Q, nprobe=NPROBE, k=80), Dr, Ir)
    assert h.cache_stats()["evictions"] > 0
    # and back to the screen
    assert_same(*h.search(Q, nprobe=NPROBE, k=10), *o.search(Q, NPROBE, 10))


def test_screened_tier_file_home_overflow_reruns(tmp_path):
    """A candidate buffer too small for a batch: the file home cannot recompute a pair over
    its whole list on the device, so the batch is re-run with a larger buffer."""
    dim = 64
    X, Q, ids, o = data(dim, seed=3)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "index.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    h.set_option("list_cache_bytes", (need_blocks(o, Q, NPROBE) + 8) * block_bytes(dim))
    h.open_lists(path)
    h.set_option("screen_cand_cap", 1024)
    h.set_batch(256)
    assert_same(*h.search(Q, nprobe=NPROBE, k=10), *o.search(Q, NPROBE, 10))
    assert h.cache_stats()["screen_reruns"] > 0


def test_screened_tier_empty_lists_stale_slots(tmp_path):
    """Reference quirk A1 (an empty probed list keeps the previous query's slot) through the
    screened tier, host and file homes, across batch boundaries."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3000, 64)).astype(np.float32)
    Q = rng.standard_normal((300, 64)).astype(np.float32)
    ids = np.arange(3000, dtype=np.uint64)
    C = np.concatenate([X[:10], 6.0 + rng.standard_normal((6, 64)).astype(np.float32) * 0.1])
    C[10:] *= np.where(rng.random((6, 1)) < 0.5, -1, 1).astype(np.float32)
    o = oracle.OracleIndex(64, 16, 0)
    o.centroids = C
    o.add(X, ids)
    assert any(o.list_count(l) == 0 for l in range(16))
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 16))
    g.centroids = C
    g.add(X, ids)
    g.set_option("list_cache_bytes", 8 * block_bytes(64))
    Dr, Ir = o.search(Q, 12, 8)
    for batch in (256, 7):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=12, k=8), Dr, Ir)
    path = str(tmp_path / "stale.vdb")
    g.save(path)
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 16))
    h.set_option("list_cache_bytes", 8 * block_bytes(64))
    h.open_lists(path)
    for batch in (256, 7):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=12, k=8), Dr, Ir)
    assert h.cache_stats()["screen_batches"] > 0


def test_screened_tier_attach_comm_world1_file_home(tmp_path):
    """A file-home screened tier with an attached communicator (world 1): per-call exchange."""
    dim = 64
    X, Q, ids, o = data(dim, seed=21)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "index.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    h.set_option("list_cache_bytes", (need_blocks(o, Q, NPROBE) + 8) * block_bytes(dim))
    h.open_lists(path)
    h.attach_comm(vdb.comm_unique_id(), 0, 1)
    for batch in (256, 33):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=NPROBE, k=10), *o.search(Q, NPROBE, 10))
    assert_same(*h.search(Q, nprobe=NPROBE, k=70), *o.search(Q, NPROBE, 70))  # the list cache
    st = h.cache_stats()
    assert st["screen_batches"] > 0 and st["evictions"] > 0, st
    h.detach_comm()


@pytest.mark.parametrize("home", ["host", "file"])
def test_screened_tier_k64_32_query_items(tmp_path, home):
    """k = 64 with nprobe >= 64 (32-query items chosen automatically) and with screen_group =
    32: the tier's routing and the batch agree that the screen serves them, so no batch
    falls to the exact scan over a cache that does not hold its lists."""
    from test_gpu_bounded import lists_pair
    dim, nlist = 64, 80
    rng = np.random.default_rng(64)
    X = rng.standard_normal((16000, dim)).astype(np.float32)
    Q = rng.standard_normal((130, dim)).astype(np.float32)
    ids = np.arange(len(X), dtype=np.uint64)
    C = rng.standard_normal((nlist, dim)).astype(np.float32)
    lists = rng.integers(0, nlist, len(X))
    g, o = lists_pair(X, ids, lists, C, 0)
    cache = 24 * block_bytes(dim)  # (a fraction of the lists: the exact path would need the cache)
    if home == "host":
        h = g
        h.set_option("list_cache_bytes", cache)
    else:
        path = str(tmp_path / "k64.vdb")
        g.save(path)
        del g
        h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist))
        h.set_option("list_cache_bytes", cache)
        h.open_lists(path)
    for nprobe, sg in ((64, 0), (70, 0), (8, 32), (64, 32), (8, 16)):
        h.set_option("screen_group", sg)
        Dr, Ir = o.search(Q, nprobe, 64)
        b0 = h.cache_stats()["screen_batches"]
        for batch in (128, 37):
            h.set_batch(batch)
            assert_same(*h.search(Q, nprobe=nprobe, k=64), Dr, Ir)
        assert h.cache_stats()["screen_batches"] > b0, (nprobe, sg)


def test_screened_tier_cancellation_falls_back_to_the_list_cache(tmp_path):
    """File home, the cancellation regime (the bound wider than the whole distance spread:
    every pair a candidate): a batch whose candidates would need a buffer above
    tier_cand_max is served by the exact list-cache path instead of growing the buffer
    without bound; results stay bit-identical."""
    from test_gpu_bounded import lists_pair
    rng = np.random.default_rng(11)
    dim = 64
    c = (100.0 / np.sqrt(dim)) * np.ones(dim, np.float32)
    X = (c + 0.01 * rng.standard_normal((12000, dim))).astype(np.float32)
    Q = (c + 0.01 * rng.standard_normal((96, dim))).astype(np.float32)
    lists = (rng.random(12000) >= 0.8).astype(np.int64)
    ids = np.arange(12000, dtype=np.uint64)
    C = np.stack([np.zeros_like(c), -c]).astype(np.float32)
    g, o = lists_pair(X, ids, lists, C, 0)
    path = str(tmp_path / "cancel.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, 2))
    h.set_option("list_cache_bytes", 200 * block_bytes(dim))
    h.open_lists(path)
    h.set_option("tier_row_cache", 0)
    h.set_option("screen_cand_cap", 1024)
    h.set_option("tier_cand_max", 4096)
    Dr, Ir = o.search(Q, 2, 10)
    for batch in (96, 40):
        h.set_batch(batch)
        assert_same(*h.search(Q, nprobe=2, k=10), Dr, Ir)
    st = h.cache_stats()
    assert st["screen_fallbacks"] > 0 and st["subbatches"] > 0, st
    # a cap the batch fits under: re-run with a larger buffer instead
    h.set_option("tier_cand_max", 1 << 24)
    f0 = st["screen_fallbacks"]
    assert_same(*h.search(Q, nprobe=2, k=10), Dr, Ir)
    st = h.cache_stats()
    assert st["screen_fallbacks"] == f0 and st["screen_reruns"] > 0, st


def test_screened_tier_row_cache_by_survivor_histogram(tmp_path):
    """The row cache refilled by the survivor rows served batches needed per list
    (vdb_ivf_survivor_histogram -> vdb_ivf_fill_row_cache), and back to the size order:
    results unchanged, survivor rows served from the cache."""
    dim = 64
    X, Q, ids, o = data(dim, seed=17)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    g.centroids = o.centroids
    g.add(X, ids)
    path = str(tmp_path / "hist.vdb")
    g.save(path)
    del g
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, NLIST))
    h.set_option("list_cache_bytes", (need_blocks(o, Q, NPROBE) + 8) * block_bytes(dim))
    h.open_lists(path)
    Dr, Ir = o.search(Q, NPROBE, 10)
    assert_same(*h.search(Q, nprobe=NPROBE, k=10), Dr, Ir)
    hist = h.survivor_histogram()
    st = h.cache_stats()
    # (every survivor counted; a row read once for several queries is fetched once)
    assert hist.sum() >= st["screen_rows_fetched"] + st["screen_rows_cached"] > 0, (hist.sum(), st)
    for w in (hist, None):
        h.fill_row_cache(w)
        s0 = h.cache_stats()
        assert_same(*h.search(Q, nprobe=NPROBE, k=10), Dr, Ir)
        s1 = h.cache_stats()
        assert s1["screen_rows_cached"] > s0["screen_rows_cached"], (s0, s1)
