"""GPU parity at BASELINE.json configs[2] and configs[3] full size (ids and distance bits).

* cfg3 — 10M x 768, nlist 4096, nprobe 32, batch 64, k 10: the bench's own index (device
  data seed 12345, train on the first 100K vectors, add all 10M) and two batches of 64
  queries searched concurrently on two streams (two workspace slots in flight, the bench's
  mode). Hub lists of ~44K vectors, wide and narrow items, segment auto-sizing and the
  fused persistent scan all run at their real shape. The oracle (ivf_flat_index.cpp:205-256
  restated) gets the GPU's centroids and every probed list; each search_device call is one
  reference search() call.
* cfg4 — 100M x 768, nlist 16384, nprobe 64 over 8 GPUs (307 GB in total, too large for
  one GPU): exact assignment of all 100M rows, the LPT plan from the final list sizes, and
  EVERY rank's shard built in turn (append of its owned lists only), its partial results
  against oracle_search_shard (owned lists scanned, the others kept as counts for the
  empty-list rule, cpp:225), then the device merge of the 8 rank records against the
  oracle's merge: the whole configuration's answer for four queries.
"""
import numpy as np
import pytest

import oracle
from conftest import load_vdb

vdb = load_vdb()
pytestmark = pytest.mark.gpu
THREADS = 16  # the GPU box's CPU share


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _export_probed(g, o, Q, nprobe, owned=None):
    """Give the oracle every list the queries probe (others: counts only)."""
    sizes = g.list_sizes()
    probed = {int(l) for qv in Q for l in o.select_nprobe(qv, nprobe)}
    for l in range(len(sizes)):
        if l in probed and (owned is None or owned[l]) and sizes[l]:
            v, i = o.list_buffers(l, int(sizes[l]))
            g.get_list_into(l, v, i)
        elif owned is not None:
            o.set_list_count(l, int(sizes[l]))
    return sizes


@pytest.mark.timeout(900)
def test_cfg3_10m_x_768_nlist4096_nprobe32_two_batches_in_flight():
    import torch
    n, dim, nlist, nprobe, B, k = 10_000_000, 768, 4096, 32, 64, 10
    dev = torch.device("cuda", 0)
    s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with torch.cuda.stream(s0):
        s = s0.cuda_stream
        data = torch.empty((n, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(data.data_ptr(), n * dim, seed=12345, stream=s)
        ids = torch.arange(n, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0))
        g.train_device(data.data_ptr(), 100_000)
        g.add_device(data.data_ptr(), ids.data_ptr(), n)
        del data, ids
        torch.cuda.empty_cache()
        q = torch.empty((2 * B, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(q.data_ptr(), 2 * B * dim, seed=12346, stream=s)
        od = torch.empty((2 * B, k), dtype=torch.float32, device=dev)
        oi = torch.empty((2 * B, k), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        for b, st in enumerate((s0, s1)):  # two searches in flight on two streams
            g.search_device(q[b * B:].data_ptr(), B, nprobe, k, od[b * B:].data_ptr(), oi[b * B:].data_ptr(),
                            st.cuda_stream)
        torch.cuda.synchronize()
        Q = q.cpu().numpy()
        D, I = od.cpu().numpy(), oi.cpu().numpy().view(np.uint64)
    assert int(g.list_sizes().sum()) == n
    o = oracle.OracleIndex(dim, nlist, 0)
    o.centroids = g.centroids
    _export_probed(g, o, Q, nprobe)
    for b in range(2):  # one reference search() call per search_device call
        Dr, Ir = o.search(Q[b * B:(b + 1) * B], nprobe, k, threads=THREADS)
        assert np.array_equal(I[b * B:(b + 1) * B], Ir), f"batch {b}: ids differ"
        assert np.array_equal(bits(D[b * B:(b + 1) * B]), bits(Dr)), f"batch {b}: distance bits differ"
    # gpu_vs_cpu_test.cpp:209-219 validity rules
    assert np.all(np.isfinite(D)) and np.all(D >= 0) and np.all(I < n)


@pytest.mark.timeout(900)
def test_cfg4_all_8_shards_and_final_merge_100m_x_768_nlist16384_nprobe64():
    """configs[3] whole: "100M x 768, nlist 16384, nprobe 64, lists sharded across 8 GPUs
    with the top-k merge". One exact assignment pass over the 100M rows; then, one shard
    at a time on this GPU, every rank r of the LPT plan (plan_shard + append of its rows):
    its partial results for the queries (one search call, written as its packed rank
    record) against oracle_search_shard over only that shard's probed lists (host memory
    freed before the next shard). Finally the 8 GPU records are merged on the device
    (vdb_merge_ranks_packed_device, the merge every rank runs after the all-gather) and
    compared with the oracle's merge of its 8 partials: the final cfg4 answer."""
    import torch
    n, dim, nlist, nprobe, k, world, chunk, nq = 100_000_000, 768, 16384, 64, 10, 8, 10_000_000, 4
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        s = torch.cuda.current_stream().cuda_stream
        data = torch.empty((chunk, dim), dtype=torch.float32, device=dev)
        rid = torch.empty(chunk, dtype=torch.int64, device=dev)
        asg = torch.empty(n, dtype=torch.int32, device=dev)
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0))
        vdb.gen_normal_device(data.data_ptr(), 100_000 * dim, seed=12345, offset=0, stream=s)
        torch.cuda.synchronize()
        g.train_device(data.data_ptr(), 100_000)
        for a in range(0, n, chunk):  # pass 1: exact assignment of every row
            vdb.gen_normal_device(data.data_ptr(), chunk * dim, seed=12345, offset=a * dim, stream=s)
            torch.cuda.synchronize()
            g.assign_device(data.data_ptr(), chunk, asg[a:].data_ptr())
        sizes = torch.bincount(asg, minlength=nlist).cpu().numpy().astype(np.uint64)
        cent = g.centroids
        g.close()
        q = torch.empty((nq, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(q.data_ptr(), nq * dim, seed=12346, stream=s)
        torch.cuda.synchronize()
        Q = q.cpu().numpy()
        rb = vdb.rank_record_bytes(nq, k)
        ids_off = vdb.rank_record_ids_offset(nq, k)
        records = torch.empty(world * rb, dtype=torch.uint8, device=dev)
        plan = vdb.shard_plan(sizes, world)
        o = oracle.OracleIndex(dim, nlist, 0)
        o.centroids = cent
        probed = {int(l) for qv in Q for l in o.select_nprobe(qv, nprobe)}
        del o
        oD = np.empty((world, nq, k), dtype=np.float32)
        oI = np.empty((world, nq, k), dtype=np.uint64)
        scanned = []
        for r in range(world):
            g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0))
            g.centroids = cent
            g.plan_shard(r, world, sizes)
            for a in range(0, n, chunk):  # pass 2: rank r appends its LPT lists only
                vdb.gen_normal_device(data.data_ptr(), chunk * dim, seed=12345, offset=a * dim, stream=s)
                torch.arange(a, a + chunk, dtype=torch.int64, device=dev, out=rid)
                torch.cuda.synchronize()
                g.add_to_lists_device(data.data_ptr(), rid.data_ptr(), asg[a:].data_ptr(), chunk)
            assert np.array_equal(g.list_sizes(), sizes)
            owned = plan == r
            assert np.array_equal(g.list_owners() == r, owned)
            rec = records[r * rb:]
            g.search_device(q.data_ptr(), nq, nprobe, k, rec.data_ptr(), rec.data_ptr() + ids_off, s)
            torch.cuda.synchronize()
            Dg = rec[:nq * k * 4].cpu().numpy().view(np.float32).reshape(nq, k)
            Ig = rec[ids_off:ids_off + nq * k * 8].cpu().numpy().view(np.uint64).reshape(nq, k)
            o = oracle.OracleIndex(dim, nlist, 0)
            o.centroids = cent
            loaded = 0
            for l in range(nlist):
                if l in probed and owned[l] and sizes[l]:
                    v, i = o.list_buffers(l, int(sizes[l]))
                    g.get_list_into(l, v, i)
                    loaded += int(sizes[l])
                else:
                    o.set_list_count(l, int(sizes[l]))
            Dr, Ir = o.search_shard(Q, nprobe, k, owned.astype(np.uint8), threads=THREADS)
            del o
            g.close()
            torch.cuda.empty_cache()
            assert np.array_equal(Ig, Ir), f"rank {r}: ids differ"
            assert np.array_equal(bits(Dg), bits(Dr)), f"rank {r}: distance bits differ"
            oD[r], oI[r] = Dr, Ir
            scanned.append(loaded)
        del data, rid, asg
        torch.cuda.empty_cache()
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        vdb.merge_ranks_packed_device(records.data_ptr(), world, nq, k, od.data_ptr(), oi.data_ptr(), s)
        torch.cuda.synchronize()
        D, I = od.cpu().numpy(), oi.cpu().numpy().view(np.uint64)
    Df, If = oracle.merge_ranks(oD, oI, k)
    assert np.array_equal(I, If), "final (merged) ids differ"
    assert np.array_equal(bits(D), bits(Df)), "final (merged) distance bits differ"
    assert int(sizes.sum()) == n
    assert sum(1 for x in scanned if x) >= 2, "the probed lists should span several shards"
    # gpu_vs_cpu_test.cpp:209-219 validity rules on the final answer
    assert np.all(np.isfinite(D)) and np.all(D >= 0) and np.all(I < n)
