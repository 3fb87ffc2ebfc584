"""GPU: the list-cache tier composed with list sharding (configs[4]: 1B x 768 over 8 GPUs,
more than the node's HBM, so every rank serves its own shard's lists through its own
cache; the reference's design for list streaming is engine/prefetcher.{h,cpp}), the
max_gpu_memory residency cap (ivf_flat_index.cpp:398-402), shard files, and the
communicator's deadline (non-blocking init, exchange watchdog).

Every result is compared bit for bit with the oracle (ivf_flat_index.cpp:205-256 restated),
under eviction: caches hold a few queries' lists, so calls are split into sub-batches and
lists are evicted and reloaded.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle
from conftest import ROOT, load_vdb
from test_gpu_parity import assert_same

vdb = load_vdb()
pytestmark = pytest.mark.gpu

D, NLIST, NPROBE, K = 64, 64, 8, 10
BLOCK_BYTES = 64 * (D * 4 + 8)  # one 64-vector block (dp = 64 here)


def fixture():
    X, Q, ids = oracle.reference_test_data(20000, 300, D, seed=5)
    o = oracle.OracleIndex(D, NLIST, 0)
    o.train(X[:5000])
    o.add(X, ids)
    blocks = np.array([(o.list_count(l) + 63) // 64 for l in range(NLIST)])
    need = max(int(blocks[o.select_nprobe(q, NPROBE)].sum()) for q in Q)  # one query's probed lists
    return X, Q, ids, o, blocks, need


def check_tier_stats(g, screen, o, Q, exact_k=100):
    """With the screen, k <= 64 searches keep the shadow resident and load no list; a k > 64
    search on the same handle then runs the list-cache path under eviction. Without it, the
    searches above already split into sub-batches and evicted."""
    st = g.cache_stats()
    if screen:
        assert st["screen_resident"] == 1 and st["screen_batches"] > 0 and st["loads"] == 0, st
        assert_same(*g.search(Q, nprobe=NPROBE, k=exact_k), *o.search(Q, NPROBE, exact_k))
        st = g.cache_stats()
    assert st["evictions"] > 0 and st["subbatches"] > 1, st


@pytest.mark.parametrize("screen", [1, 0], ids=["screened", "list-cache"])
def test_tier_with_attached_communicator_under_eviction(screen):
    """A tiered handle with an RCCL communicator (world 1): each call's partials go into one
    record, ONE all-gather per call, the merge; results equal the oracle whatever the cache
    holds. The tier may be switched on before or after attach_comm."""
    import torch
    X, Q, ids, o, blocks, need = fixture()
    Dr, Ir = o.search(Q, NPROBE, K)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
    g.set_option("screen", screen)
    g.centroids = o.centroids
    g.add(X, ids)
    g.set_option("list_cache_bytes", (need + 8) * BLOCK_BYTES)  # before attach
    g.attach_comm(vdb.comm_unique_id(), 0, 1)
    for batch in (256, 16, 1):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    check_tier_stats(g, screen, o, Q)
    import time
    t0 = time.time()
    while True:  # (the watchdog polls completions: its count may trail the host by a moment)
        err, issued, done = g.comm_status()
        if done == issued or time.time() - t0 > 5:
            break
        time.sleep(0.01)
    assert err is None and issued >= 3 and done == issued, (err, issued, done)
    # device API on two streams in flight
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(Q).to(dev)
    od = torch.empty((300, K), dtype=torch.float32, device=dev)
    oi = torch.empty((300, K), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for j, s in enumerate(streams):
        g.search_device(q[j * 150:].data_ptr(), 150, NPROBE, K, od[j * 150:].data_ptr(), oi[j * 150:].data_ptr(),
                        s.cuda_stream)
    torch.cuda.synchronize()
    for j in range(2):
        assert_same(od[j * 150:(j + 1) * 150].cpu().numpy(), oi[j * 150:(j + 1) * 150].cpu().numpy().view(np.uint64),
                    *o.search(Q[j * 150:(j + 1) * 150], NPROBE, K))
    # tier off and on again while attached (the plain per-batch exchange in between)
    g.set_option("list_cache_bytes", 0)
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    g.set_option("list_cache_bytes", (2 * need + 8) * BLOCK_BYTES)
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    g.detach_comm()
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)


def test_tiered_shard_with_communicator_every_list_cached():
    """A tiered handle whose cache holds every stored list takes the plain batches but
    still one exchange per call (all ranks must issue the same collectives)."""
    X, Q, ids, o, blocks, need = fixture()
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
    g.centroids = o.centroids
    g.add(X, ids)
    g.attach_comm(vdb.comm_unique_id(), 0, 1)
    g.set_option("list_cache_bytes", int(blocks.sum() + 4) * BLOCK_BYTES)  # after attach
    g.warmup_lists(list(range(NLIST)))
    g.set_batch(64)
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), *o.search(Q, NPROBE, K))
    assert g.cache_stats()["subbatches"] == 0  # everything cached: no tier sub-batches


@pytest.mark.parametrize("screen", [1, 0], ids=["screened", "list-cache"])
@pytest.mark.parametrize("stale", [False, True])
def test_tiered_group_two_members_one_device_under_eviction(stale, screen):
    """A 2-member group on one device whose members serve their lists through their own
    list caches: one record per member for the whole call, one exchange, the merge."""
    if stale:  # empty probed lists (reference quirk A1) across sub-batches and members
        rng = np.random.default_rng(0)
        X = rng.standard_normal((3000, 16)).astype(np.float32)
        Q = rng.standard_normal((300, 16)).astype(np.float32)
        ids = np.arange(3000, dtype=np.uint64)
        C = np.concatenate([X[:10], 6.0 + rng.standard_normal((6, 16)).astype(np.float32) * 0.1])
        C[10:] *= np.where(rng.random((6, 1)) < 0.5, -1, 1).astype(np.float32)
        o = oracle.OracleIndex(16, 16, 0)
        o.centroids = C
        o.add(X, ids)
        dim, nlist, nprobe, k = 16, 16, 12, 8
        blocks = np.array([(o.list_count(l) + 63) // 64 for l in range(nlist)])
        cap = (int(np.sort(blocks)[::-1][:6].sum()) + 2) * 64 * (64 * 4 + 8)
    else:
        X, Q, ids, o, blocks, need = fixture()
        dim, nlist, nprobe, k = D, NLIST, NPROBE, K
        C = o.centroids
        cap = (need + 8) * BLOCK_BYTES
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0, devices=(0, 0)))
    g.set_option("screen", screen)
    g.centroids = C
    g.add(X, ids)
    g.set_option("list_cache_bytes", cap)  # per member
    Dr, Ir = o.search(Q, nprobe, k)
    for batch in (256, 7):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=nprobe, k=k), Dr, Ir)
    st = g.cache_stats()  # summed over the members
    if screen:  # the shadow of both members resident, no list loaded; k > 64: the list caches
        assert st["screen_resident"] == 1 and st["screen_batches"] > 0 and st["loads"] == 0, st
        assert_same(*g.search(Q, nprobe=nprobe, k=100), *o.search(Q, nprobe, 100))
        st = g.cache_stats()
    assert st["capacity_bytes"] > 0 and st["loads"] > 0 and st["subbatches"] > 0, st
    g.warmup_lists([0, 1])
    g.evict_list(0)
    assert_same(*g.search(Q, nprobe=nprobe, k=k), Dr, Ir)


@pytest.mark.parametrize("screen", [1, 0], ids=["screened", "list-cache"])
def test_shard_files_served_per_rank(tmp_path, screen):
    """configs[4]'s deployment on one GPU: each rank of an LPT shard plan saves a SHARD
    file (every list's count, only its own lists' rows); a fresh handle serves that file
    through its cache and becomes that rank's shard (rank and world from the file). Each
    rank's partial results equal the oracle's shard search, and the merge of the ranks'
    records equals the oracle's full search."""
    import torch
    X, Q, ids, o, blocks, need = fixture()
    world = 3
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(Q).to(dev)
    n = len(Q)
    rb = vdb.rank_record_bytes(n, K)
    recs = torch.empty(world * rb, dtype=torch.uint8, device=dev)
    sizes = None
    for r in range(world):
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
        g.centroids = o.centroids
        g.add(X, ids)
        sizes = g.list_sizes()
        g.set_shard(r, world)
        path = str(tmp_path / f"shard{r}.ivf")
        g.save(path)  # a sharded handle writes a shard file
        assert os.path.getsize(path) < 24 + NLIST * D * 4 + NLIST * 16 + len(X) * (8 + D * 4)
        Dp, Ip = g.search(Q, nprobe=NPROBE, k=K)
        del g
        h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
        h.set_option("screen", screen)
        h.set_option("list_cache_bytes", (need + 8) * BLOCK_BYTES)
        h.open_lists(path)
        owners = h.list_owners()
        owned = vdb.shard_plan(sizes, world) == r
        assert np.all((owners == r)[sizes > 0] == owned[sizes > 0])
        h.set_batch(16)
        Dh, Ih = h.search(Q, nprobe=NPROBE, k=K)
        assert_same(Dh, Ih, Dp, Ip)
        assert_same(Dh, Ih, *o.search_shard(Q, NPROBE, K, owned.astype(np.uint8)))
        st = h.cache_stats()
        assert st["file_bytes_read"] > 0
        if screen:  # the file streamed once (the shadow), then only the survivors' rows
            # (the idle cache holds the largest lists: their survivors are copied from HBM)
            assert st["screen_rows_fetched"] + st["screen_rows_cached"] > 0, st
            probed = sum(int(sizes[l]) for q in Q for l in o.select_nprobe(q, NPROBE) if owned[l])
            assert st["screen_rows_fetched"] + st["screen_rows_cached"] < 0.25 * probed, (st, probed)
        with pytest.raises(vdb.VdbError):
            h.set_shard((r + 1) % world, world)  # the file holds only this rank's lists
        s = torch.cuda.Stream(dev)
        rec = recs[r * rb:]
        h.search_device(q.data_ptr(), n, NPROBE, K, rec.data_ptr(), rec.data_ptr() + vdb.rank_record_ids_offset(n, K),
                        s.cuda_stream)
        torch.cuda.synchronize()
        single = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
        with pytest.raises(vdb.VdbError, match="shard file"):
            single.load(path)
    od = torch.empty((n, K), dtype=torch.float32, device=dev)
    oi = torch.empty((n, K), dtype=torch.int64, device=dev)
    vdb.merge_ranks_packed_device(recs.data_ptr(), world, n, K, od.data_ptr(), oi.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert_same(od.cpu().numpy(), oi.cpu().numpy().view(np.uint64), *o.search(Q, NPROBE, K))


@pytest.mark.parametrize("screen", [1, 0], ids=["screened", "list-cache"])
def test_max_gpu_memory_caps_list_residency(screen):
    """Config::max_gpu_memory (the reference's cap on resident list bytes): an index that
    outgrows it is served through the list-cache tier with an HBM cache of that size,
    results unchanged; 0 = no cap; a cap below one query's lists fails the search with
    VDB_ERR_OUT_OF_MEMORY (the reference would search such lists on the CPU)."""
    X, Q, ids, o, blocks, need = fixture()
    Dr, Ir = o.search(Q, NPROBE, K)
    cap = (2 * need + 8) * BLOCK_BYTES
    assert cap < len(X) * (D * 4 + 8)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=cap))
    g.set_option("screen", screen)
    g.centroids = o.centroids
    g.add(X[:100], ids[:100])
    assert g.cache_stats()["capacity_bytes"] == 0  # still under the cap: every list in HBM
    g.add(X[100:], ids[100:])
    st = g.cache_stats()
    assert st["capacity_bytes"] == (cap // BLOCK_BYTES) * BLOCK_BYTES
    # (the footprint also counts the search workspaces: a small allowance)
    assert g.gpu_bytes_allocated() <= cap + (NLIST * 64 * 4 * 2) + BLOCK_BYTES + (1 << 20)
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    check_tier_stats(g, screen, o, Q)
    # the cap lifted: the lists return to HBM
    g.set_option("max_gpu_memory", 0)
    assert g.cache_stats()["capacity_bytes"] == 0
    assert_same(*g.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    # no cap
    h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
    h.centroids = o.centroids
    h.add(X, ids)
    assert h.cache_stats()["capacity_bytes"] == 0
    # a cap below one query's lists
    t = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=max(need // 2, 1) * BLOCK_BYTES))
    t.set_option("screen", screen)
    t.centroids = o.centroids
    t.add(X, ids)
    if screen:  # the screened tier loads no list: the small cache does not matter for k <= 64
        assert_same(*t.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    with pytest.raises(vdb.VdbError) as ei:
        t.search(Q, nprobe=NPROBE, k=100 if screen else K)
    assert ei.value.code == -3
    # the option form applies at once
    h.set_option("max_gpu_memory", cap)
    assert h.cache_stats()["capacity_bytes"] == (cap // BLOCK_BYTES) * BLOCK_BYTES
    assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)
    # the cap raised above the lists: back to HBM
    h.set_option("max_gpu_memory", 10 * len(X) * (D * 4 + 8))
    assert h.cache_stats()["capacity_bytes"] == 0
    assert_same(*h.search(Q, nprobe=NPROBE, k=K), Dr, Ir)


def test_result_changing_diagnostics_are_not_options():
    """Timing experiments that invalidate results exist only as separate builds
    (VDB_SCAN_DIAG); the runtime options never change results."""
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(16, 4))
    with pytest.raises(vdb.VdbError, match="unknown option"):
        g.set_option("diag", 1)
    g.set_option("bounded_stats", 1)
    g.set_option("comm_timeout_ms", 5000)
    assert len(vdb.build_id()) == 16


_COMM_SCRIPT = textwrap.dedent(r"""
    import ctypes, json, sys, time
    sys.path.insert(0, sys.argv[1])
    sys.path.insert(0, sys.argv[1] + "/tests")
    from conftest import load_vdb
    import numpy as np
    import torch
    vdb = load_vdb()
    out = {}
    X = np.random.default_rng(0).standard_normal((2000, 16)).astype(np.float32)
    ids = np.arange(2000, dtype=np.uint64)
    Q = X[:50].copy()
    mode = sys.argv[2]
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(16, 8, max_gpu_memory=0))
    g.train(X)
    g.add(X, ids)
    D0, I0 = g.search(Q, nprobe=4, k=5)
    if mode == "init":
        # world 2 with no second rank: the non-blocking init must end at the deadline
        g.set_shard(0, 2)
        D0, I0 = g.search(Q, nprobe=4, k=5)  # this shard's partial results
        g.set_option("comm_timeout_ms", 3000)
        t0 = time.time()
        try:
            g.attach_comm(vdb.comm_unique_id(), 0, 2)
            out["raised"] = False
        except vdb.VdbError as e:
            out["raised"], out["msg"], out["code"] = True, str(e), e.code
        out["seconds"] = time.time() - t0
        D1, I1 = g.search(Q, nprobe=4, k=5)  # the handle still serves (no communicator)
        out["after_ok"] = bool(np.array_equal(I0, I1))
    else:
        # world 1, the caller's stream held back by a wait on a signal: the exchange cannot
        # complete, the watchdog must report it after the deadline; then the stream is
        # released and the exchange completes; later searches fail until detach
        # the HIP runtime torch (and the engine) already use, not a second copy
        path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
        hip = ctypes.CDLL(path)
        g.set_option("comm_timeout_ms", 1500)
        g.attach_comm(vdb.comm_unique_id(), 0, 1)
        sig = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(sig), ctypes.c_size_t(8), ctypes.c_uint(2)) == 0  # hipMallocSignalMemory
        assert hip.hipMemset(sig, 0, ctypes.c_size_t(8)) == 0
        assert hip.hipDeviceSynchronize() == 0
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        rel = torch.cuda.Stream(dev)
        rc = hip.hipStreamWaitValue32(ctypes.c_void_p(s.cuda_stream), sig, ctypes.c_uint32(1), ctypes.c_uint(0),
                                      ctypes.c_uint32(0xFFFFFFFF))  # hipStreamWaitValueGte
        out["wait_rc"] = rc
        q = torch.from_numpy(Q).to(dev)
        od = torch.empty((50, 5), dtype=torch.float32, device=dev)
        oi = torch.empty((50, 5), dtype=torch.int64, device=dev)
        try:
            g.search_device(q.data_ptr(), 50, 4, 5, od.data_ptr(), oi.data_ptr(), s.cuda_stream)
            t0 = time.time()
            err = None
            while time.time() - t0 < 20 and err is None:
                err, issued, done = g.comm_status()
                time.sleep(0.05)
            out["watchdog_s"] = time.time() - t0
            out["err"] = err
        finally:
            hip.hipStreamWriteValue32(ctypes.c_void_p(rel.cuda_stream), sig, ctypes.c_uint32(1), ctypes.c_uint(0))
            torch.cuda.synchronize()
        out["released_ok"] = bool(np.array_equal(oi.cpu().numpy().view(np.uint64), I0))
        try:
            g.search(Q, nprobe=4, k=5)
            out["after_raised"] = False
        except vdb.VdbError:
            out["after_raised"] = True
        g.detach_comm()
        D1, I1 = g.search(Q, nprobe=4, k=5)
        out["after_detach_ok"] = bool(np.array_equal(I0, I1))
    print("RESULT " + json.dumps(out), flush=True)
""")


def _run_comm_script(mode):
    p = subprocess.run([sys.executable, "-c", _COMM_SCRIPT, ROOT, mode], capture_output=True, text=True, timeout=150)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-2000:]
    import json
    return json.loads(lines[-1][7:])


def test_comm_init_deadline_names_the_rank():
    """Non-blocking communicator init: a peer that never joins ends attach_comm at the
    deadline with VDB_ERR_DEVICE naming this rank (no hang), and the handle keeps serving."""
    r = _run_comm_script("init")
    assert r["raised"] and r["code"] == -2, r
    assert "rank 0 of 2" in r["msg"], r
    assert r["seconds"] < 60, r
    assert r["after_ok"], r


def test_exchange_watchdog_reports_a_stalled_exchange():
    """An exchange that cannot complete (its stream held back) is reported by the watchdog
    after comm_timeout_ms, naming the rank; released, it completes with correct results;
    the communicator stays failed until detached."""
    r = _run_comm_script("exchange")
    if r.get("wait_rc", 0) != 0:
        pytest.skip(f"hipStreamWaitValue32 unavailable (rc {r['wait_rc']})")
    assert r["err"] and "rank 0 of 1" in r["err"] and "exchange" in r["err"], r
    assert 1.0 < r["watchdog_s"] < 15, r
    assert r["released_ok"] and r["after_raised"] and r["after_detach_ok"], r


def test_probe_census_and_weighted_plan_shards():
    """vdb_ivf_probe_census equals the oracle's probe histogram (select_nprobe on the same
    rows); shards cut by the probe-weighted plan (explicit owners) merge to the oracle's
    full answer."""
    import torch
    X, Q, ids, o, blocks, need = fixture()
    dev = torch.device("cuda", 0)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
    g.centroids = o.centroids
    g.add(X, ids)
    rows = torch.from_numpy(X[:3000]).to(dev)
    counts = g.probe_census(rows.data_ptr(), 3000, NPROBE)
    ref = np.zeros(NLIST, dtype=np.uint64)
    for x in X[:3000]:
        ref[o.select_nprobe(x, NPROBE)] += 1
    assert np.array_equal(counts, ref)
    sizes = g.list_sizes()
    world = 3
    owners = vdb.shard_plan_probe_weighted(sizes, counts, 3000, 64, world)
    n = len(Q)
    rb = vdb.rank_record_bytes(n, K)
    recs = torch.empty(world * rb, dtype=torch.uint8, device=dev)
    q = torch.from_numpy(Q).to(dev)
    for r in range(world):
        h = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
        h.centroids = o.centroids
        h.add(X, ids)
        h.set_shard(r, world, owners=owners)
        assert np.array_equal(h.list_owners() == r, owners == r)
        s = torch.cuda.Stream(dev)
        rec = recs[r * rb:]
        h.search_device(q.data_ptr(), n, NPROBE, K, rec.data_ptr(), rec.data_ptr() + vdb.rank_record_ids_offset(n, K),
                        s.cuda_stream)
        torch.cuda.synchronize()
    od = torch.empty((n, K), dtype=torch.float32, device=dev)
    oi = torch.empty((n, K), dtype=torch.int64, device=dev)
    vdb.merge_ranks_packed_device(recs.data_ptr(), world, n, K, od.data_ptr(), oi.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert_same(od.cpu().numpy(), oi.cpu().numpy().view(np.uint64), *o.search(Q, NPROBE, K))


def test_queries_read_in_place_and_misaligned():
    """dim a multiple of 64 (the padded width): the kernels read the caller's query rows in
    place (no padding copy); a pointer that is not 16-byte aligned falls back to the
    padded copy. Both equal the oracle, fused and unfused merges alike."""
    import torch
    X, Q, ids, o, blocks, need = fixture()
    Dr, Ir = o.search(Q, NPROBE, K)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(D, NLIST, max_gpu_memory=0))
    g.centroids = o.centroids
    g.add(X, ids)
    dev = torch.device("cuda", 0)
    n = len(Q)
    buf = torch.zeros(n * D + 1, dtype=torch.float32, device=dev)
    od = torch.empty((n, K), dtype=torch.float32, device=dev)
    oi = torch.empty((n, K), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    for fm in (1, 0):
        g.set_option("fused_merge", fm)
        for off in (0, 1):  # 16-byte aligned rows, then rows 4 bytes off
            buf[off:off + n * D] = torch.from_numpy(Q.reshape(-1)).to(dev)
            torch.cuda.synchronize()
            g.search_device(buf.data_ptr() + 4 * off, n, NPROBE, K, od.data_ptr(), oi.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            assert_same(od.cpu().numpy(), oi.cpu().numpy().view(np.uint64), Dr, Ir)

