"""GPU tests of the multi-GPU search path inside the engine (group.cpp and
the exchange in engine.hpp): the per-batch packed partial records, the RCCL all-gather and
the on-device merge, against the oracle (ivf_flat_index.cpp:205-256 restated).

The GPU box has one MI355X, so:
* the RCCL path runs at world size 1 — a communicator attached to a handle
  (ncclCommInitRank, one process per GPU) and a group over one device
  (ncclCommInitAll) — which executes the same broadcast / all-gather / merge code;
* the N-member semantics (list placement, per-member partials with stale-slot sources,
  the merge of N records) run on groups whose members share the one device and exchange
  through device copies. RCCL itself wants one rank per GPU; the driver's 8-GPU node
  runs the N-rank RCCL path (bench.py --gpus N).
"""
import threading

import numpy as np
import pytest

import oracle
from conftest import load_vdb

vdb = load_vdb()
pytestmark = pytest.mark.gpu
NONE = np.iinfo(np.uint32).max


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_same(D, I, Dr, Ir):
    assert I.shape == Ir.shape
    bad = np.argwhere(I != Ir)
    assert bad.size == 0, f"ids differ at {bad[:5].tolist()}"
    assert np.array_equal(bits(D), bits(Dr)), "distance bits differ"


def ctest_data():
    return oracle.reference_test_data(10000, 100, 64)  # gpu_vs_cpu_test ctest args 10000 100 64 32


def stale_fixture():
    """Data whose probed lists include empty ones (reference quirk A1, cpp:210-233)."""
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
    return X, Q, ids, C, o


def test_attached_communicator_world1_rccl():
    X, Q, ids = ctest_data()
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, ids)
    Dr, Ir = o.search(Q, 8, 10)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32))
    g.train(X)
    g.add(X, ids)
    with pytest.raises(vdb.VdbError):
        g.attach_comm(vdb.comm_unique_id(), 0, 2)  # the handle's shard is (0, 1)
    g.attach_comm(vdb.comm_unique_id(), 0, 1)   # ncclCommInitRank: records all-gathered per batch
    for batch in (7, 256):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=8, k=10), Dr, Ir)
    import torch
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(Q).to(dev)
    od = torch.empty((100, 10), dtype=torch.float32, device=dev)
    oi = torch.empty((100, 10), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    g.search_device(q.data_ptr(), 100, 8, 10, od.data_ptr(), oi.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    assert_same(od.cpu().numpy(), oi.cpu().numpy().view(np.uint64), Dr, Ir)
    g.detach_comm()
    assert_same(*g.search(Q, nprobe=8, k=10), Dr, Ir)


def test_group_one_device_rccl():
    X, Q, ids = ctest_data()
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, ids)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32, devices=(0,)))
    assert g.group_size == 1
    g.train(X)
    assert np.array_equal(bits(g.centroids), bits(o.centroids))
    g.add(X, ids)
    assert np.all(g.list_owners()[g.list_sizes() > 0] == 0)
    assert_same(*g.search(Q, nprobe=8, k=10), *o.search(Q, 8, 10))


@pytest.mark.parametrize("members", [2, 3])
def test_group_members_sharing_one_device(members, tmp_path):
    X, Q, ids = ctest_data()
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, ids)
    Dr, Ir = o.search(Q, 8, 10)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32, devices=(0,) * members))
    assert g.group_size == members
    g.train(X)
    assert np.array_equal(bits(g.centroids), bits(o.centroids)), "train() on a group differs"
    g.add(X, ids)
    sizes = g.list_sizes()
    assert g.get_total_vectors() == 10000 and int(sizes.sum()) == 10000
    owners = g.list_owners()
    # a bulk add places lists exactly as the LPT plan of the one-process-per-GPU path
    assert np.array_equal(owners[sizes > 0], vdb.shard_plan(sizes, members)[sizes > 0])
    assert len(set(owners[sizes > 0].tolist())) == members
    for l in range(32):
        gv, gi = g.get_list(l)
        ov, oi = o.get_list(l)
        assert np.array_equal(gi, oi) and np.array_equal(bits(gv), bits(ov))
    for batch in (7, 256):
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=8, k=10), Dr, Ir)
    assert g.get_gpu_memory_usage() == 10000 * (64 * 4 + 8)   # count * (dim * 4 + 8), summed over members
    # device API: queries and results on the group's first device
    import torch
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(Q).to(dev)
    od = torch.empty((100, 10), dtype=torch.float32, device=dev)
    oi = torch.empty((100, 10), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for j, s in enumerate(streams):  # two calls in flight
        g.search_device(q[j * 50:].data_ptr(), 50, 8, 10, od[j * 50:].data_ptr(), oi[j * 50:].data_ptr(),
                        s.cuda_stream)
    torch.cuda.synchronize()
    for j in range(2):
        assert_same(od[j * 50:(j + 1) * 50].cpu().numpy(), oi[j * 50:(j + 1) * 50].cpu().numpy().view(np.uint64),
                    *o.search(Q[j * 50:(j + 1) * 50], 8, 10))
    # save from the group, load into a single-device handle and into a fresh group
    path = str(tmp_path / "group.ivf")
    g.save(path)
    single = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32))
    single.load(path)
    assert_same(*single.search(Q, nprobe=8, k=10), Dr, Ir)
    g2 = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32, devices=(0,) * members))
    g2.load(path)
    assert_same(*g2.search(Q, nprobe=8, k=10), Dr, Ir)
    with pytest.raises(vdb.VdbError):
        g2.load(path)  # load() fills an empty index only
    with pytest.raises(vdb.VdbError):
        g.set_shard(0, 2)


def test_group_stale_slots_incremental_adds_and_concurrent_calls():
    X, Q, ids, C, o = stale_fixture()
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(16, 16, devices=(0, 0, 0)))
    g.centroids = C
    for a, b in ((0, 1200), (1200, 1201), (1201, 3000)):  # lists placed as they first receive vectors
        g.add(X[a:b], ids[a:b])
    owners = g.list_owners()
    assert np.all(owners[g.list_sizes() == 0] == NONE)
    for l in range(16):
        assert np.array_equal(g.get_list(l)[1], o.get_list(l)[1])
    for batch in (7, 64, 256):  # the stale-slot carry crosses internal batches of one call
        g.set_batch(batch)
        assert_same(*g.search(Q, nprobe=12, k=8), *o.search(Q, 12, 8))
    # concurrent host calls are coalesced into shared device batches; each call keeps the
    # results it gets alone (its own probe slots)
    g.set_batch(16)
    calls = [(Q[i * 25:(i + 1) * 25], 12 if i % 2 else 9, 8 if i % 3 else 5) for i in range(12)]
    out = [None] * len(calls)

    def run(i):
        q, p, k = calls[i]
        out[i] = g.search(q, nprobe=p, k=k)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(calls))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i, (q, p, k) in enumerate(calls):
        assert_same(*out[i], *o.search(q, p, k))


def test_torch_nccl_world1_exchange():
    """bench.py's --exchange torch path: one rank's packed record all-gathered with
    torch.distributed's nccl (RCCL) backend, then vdb_merge_ranks_packed_device."""
    import torch
    import torch.distributed as dist
    X, Q, ids = ctest_data()
    o = oracle.OracleIndex(64, 32, 0)
    o.train(X)
    o.add(X, ids)
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(64, 32))
    g.centroids = o.centroids
    g.add(X, ids)
    dev = torch.device("cuda", 0)
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    st = torch.cuda.Stream(dev)
    try:
        torch.cuda.set_stream(st)  # an explicit stream: handle 0 would mean the engine's own stream
        B, k = 100, 10
        rec = vdb.rank_record_bytes(B, k)
        part = torch.empty(rec, dtype=torch.uint8, device=dev)
        gat = torch.empty(rec, dtype=torch.uint8, device=dev)
        q = torch.from_numpy(Q).to(dev)
        od = torch.empty((B, k), dtype=torch.float32, device=dev)
        oi = torch.empty((B, k), dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        g.search_device(q.data_ptr(), B, 8, k, part.data_ptr(), part.data_ptr() + vdb.rank_record_ids_offset(B, k), s)
        dist.all_gather_into_tensor(gat, part)
        vdb.merge_ranks_packed_device(gat.data_ptr(), 1, B, k, od.data_ptr(), oi.data_ptr(), s)
        torch.cuda.synchronize()
        assert_same(od.cpu().numpy(), oi.cpu().numpy().view(np.uint64), *o.search(Q, 8, 10))
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        dist.destroy_process_group()
