"""GPU parity at BASELINE.json configs[2] and configs[3] full size (ids and distance bits).

* cfg3 — 10M x 768, nlist 4096, nprobe 32, batch 64, k 10: the bench's own index (device
  data seed 12345, train on the first 100K vectors, add all 10M) and two batches of 64
  queries searched concurrently on two streams (two workspace slots in flight, the bench's
  mode). Hub lists of ~44K vectors, wide and narrow items, segment auto-sizing and the
  fused persistent scan all run at their real shape. The oracle (ivf_flat_index.cpp:205-256
  restated) gets the GPU's centroids and every probed list; each search_device call is one
  reference search() call.
  The list assignment that defines every list's contents (assign_to_lists,
  ivf_flat_index.cpp:259-295) is pinned at this shape too: 16,384 rows of the database
  re-generated on the device, assigned by the engine (MFMA bounds + exact re-check at D 768,
  nlist 4096) against the oracle's argmin row by row, and the lists that hold those rows
  compared with the oracle's membership in append order (their ids and vector bits).
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


def _window_assignment(g, o, dev, st, a, w, dim):
    """Rows [a, a + w) of the seed-12345 database re-generated on the device: the engine's
    assignment of them (vdb_ivf_assign_device) against the oracle's (cpp:259-295, strict '<'),
    row by row. Returns the rows and the oracle's lists."""
    import torch
    with torch.cuda.stream(st):
        rows = torch.empty((w, dim), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(rows.data_ptr(), w * dim, seed=12345, offset=a * dim, stream=st.cuda_stream)
        out = torch.empty(w, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        g.assign_device(rows.data_ptr(), w, out.data_ptr())
        torch.cuda.synchronize()
        R, A = rows.cpu().numpy(), out.cpu().numpy().view(np.uint32)
    Aref = o.assign(R, threads=THREADS)
    bad = np.nonzero(A != Aref)[0]
    assert bad.size == 0, f"{bad.size} of {w} rows assigned differently, first row {a + bad[0]}: gpu {A[bad[0]]} ref {Aref[bad[0]]}"
    return R, Aref


def _check_window_lists(g, R, Aref, a, lists):
    """The engine's lists in append order: the ids it stores in [a, a + len(R)) are exactly the
    window rows the oracle assigns to the list, ascending (add appends in input order,
    cpp:148-202), with the rows' vector bits."""
    for l in lists:
        v, ids = g.get_list(int(l))
        m = (ids >= a) & (ids < a + len(R))
        want = np.nonzero(Aref == l)[0].astype(np.uint64) + np.uint64(a)
        assert np.array_equal(ids[m], want), f"list {l}: window members differ or out of append order"
        assert np.array_equal(bits(v[m]), bits(R[(want - np.uint64(a)).astype(np.int64)])), f"list {l}: vector bits differ"


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
    # the assignment at full scale (D 768, nlist 4096): 16,384 rows, two windows of the database
    for a in (3_000_000, 9_000_000):
        R, Aref = _window_assignment(g, o, dev, s0, a, 8192, dim)
        lists, cnt = np.unique(Aref, return_counts=True)
        order = np.argsort(-cnt, kind="stable")
        # the lists holding most of the window's rows (the hub lists) and two of the fewest
        _check_window_lists(g, R, Aref, a, list(lists[order[:3]]) + list(lists[order[-2:]]))


CFG4 = dict(n=100_000_000, dim=768, nlist=16384, nprobe=64, k=10, world=8, chunk=10_000_000, nq=4)
_cfg4 = {}


def _cfg4_setup():
    """One exact assignment pass over the 100M rows (shared by the two cfg4 tests)."""
    if _cfg4:
        return _cfg4
    import torch
    c = CFG4
    n, dim, nlist, chunk, nq = c["n"], c["dim"], c["nlist"], c["chunk"], c["nq"]
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        s = st.cuda_stream
        data = torch.empty((chunk, dim), dtype=torch.float32, device=dev)
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
    o = oracle.OracleIndex(dim, nlist, 0)
    o.centroids = cent
    Q = q.cpu().numpy()
    _cfg4.update(dev=dev, stream=st, data=data, asg=asg, sizes=sizes, cent=cent, q=q, Q=Q,
                 plan=vdb.shard_plan(sizes, c["world"]),
                 probed={int(l) for qv in Q for l in o.select_nprobe(qv, c["nprobe"])},
                 records=torch.empty(c["world"] * vdb.rank_record_bytes(nq, c["k"]), dtype=torch.uint8, device=dev),
                 oD=np.empty((c["world"], nq, c["k"]), dtype=np.float32),
                 oI=np.empty((c["world"], nq, c["k"]), dtype=np.uint64), done=set(), scanned={})
    return _cfg4


@pytest.mark.timeout(900)
def test_cfg4_assignment_nlist16384_matches_oracle():
    """configs[3]'s list assignment, which decides every shard's contents: 4,096 rows in two
    windows of the 100M database, the engine's bulk assignment (the pass every shard's build
    uses) and a fresh vdb_ivf_assign_device of the same rows, both against the oracle's
    argmin (cpp:259-295) at nlist 16384, D 768 — where near-ties are densest."""
    import torch
    e = _cfg4_setup()
    dim, nlist = CFG4["dim"], CFG4["nlist"]
    g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0))
    g.centroids = e["cent"]
    o = oracle.OracleIndex(dim, nlist, 0)
    o.centroids = e["cent"]
    for a in (123_456, 77_777_216):
        R, Aref = _window_assignment(g, o, e["dev"], e["stream"], a, 2048, dim)
        bulk = e["asg"][a:a + 2048].cpu().numpy().view(np.uint32)
        assert np.array_equal(bulk, Aref), f"bulk assignment differs at {np.nonzero(bulk != Aref)[0][:5] + a}"
        e.setdefault("windows", []).append((a, R, Aref))
    g.close()
    torch.cuda.empty_cache()


def _cfg4_rank(r):
    """Rank r of the LPT plan built on this GPU (plan_shard + append of its rows), its packed
    rank record for the queries against oracle_search_shard over only its probed lists."""
    import torch
    c, e = CFG4, _cfg4_setup()
    if r in e["done"]:
        return
    n, dim, nlist, nprobe, k, world, chunk, nq = (c[x] for x in ("n", "dim", "nlist", "nprobe", "k", "world",
                                                                  "chunk", "nq"))
    dev, data, asg, sizes, cent = e["dev"], e["data"], e["asg"], e["sizes"], e["cent"]
    rb, ids_off = vdb.rank_record_bytes(nq, k), vdb.rank_record_ids_offset(nq, k)
    with torch.cuda.stream(e["stream"]):
        s = e["stream"].cuda_stream
        rid = torch.empty(chunk, dtype=torch.int64, device=dev)
        g = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, nlist, max_gpu_memory=0))
        g.centroids = cent
        g.plan_shard(r, world, sizes)
        for a in range(0, n, chunk):  # pass 2: rank r appends its LPT lists only
            vdb.gen_normal_device(data.data_ptr(), chunk * dim, seed=12345, offset=a * dim, stream=s)
            torch.arange(a, a + chunk, dtype=torch.int64, device=dev, out=rid)
            torch.cuda.synchronize()
            g.add_to_lists_device(data.data_ptr(), rid.data_ptr(), asg[a:].data_ptr(), chunk)
        assert np.array_equal(g.list_sizes(), sizes)
        owned = e["plan"] == r
        assert np.array_equal(g.list_owners() == r, owned)
        for a, R, Aref in e.get("windows", []):  # (this shard's lists holding rows of the windows)
            mine = [l for l in np.unique(Aref) if owned[l]]
            _check_window_lists(g, R, Aref, a, mine[:2])
        rec = e["records"][r * rb:]
        g.search_device(e["q"].data_ptr(), nq, nprobe, k, rec.data_ptr(), rec.data_ptr() + ids_off, s)
        torch.cuda.synchronize()
        Dg = rec[:nq * k * 4].cpu().numpy().view(np.float32).reshape(nq, k)
        Ig = rec[ids_off:ids_off + nq * k * 8].cpu().numpy().view(np.uint64).reshape(nq, k)
        o = oracle.OracleIndex(dim, nlist, 0)
        o.centroids = cent
        loaded = 0
        for l in range(nlist):
            if l in e["probed"] and owned[l] and sizes[l]:
                v, i = o.list_buffers(l, int(sizes[l]))
                g.get_list_into(l, v, i)
                loaded += int(sizes[l])
            else:
                o.set_list_count(l, int(sizes[l]))
        Dr, Ir = o.search_shard(e["Q"], nprobe, k, owned.astype(np.uint8), threads=THREADS)
        del o
        g.close()
        torch.cuda.empty_cache()
    assert np.array_equal(Ig, Ir), f"rank {r}: ids differ"
    assert np.array_equal(bits(Dg), bits(Dr)), f"rank {r}: distance bits differ"
    e["oD"][r], e["oI"][r] = Dr, Ir
    e["scanned"][r] = loaded
    e["done"].add(r)


@pytest.mark.timeout(900)
def test_cfg4_shards_0_to_3_100m_x_768_nlist16384_nprobe64():
    """configs[3] ("100M x 768, nlist 16384, nprobe 64, lists sharded across 8 GPUs with the
    top-k merge"), first half: one exact assignment pass over the 100M rows, then ranks 0-3
    of the LPT plan built one at a time on this GPU, each one's partial results against
    oracle_search_shard over only that shard's probed lists (host memory freed before the
    next shard)."""
    for r in range(4):
        _cfg4_rank(r)


@pytest.mark.timeout(900)
def test_cfg4_shards_4_to_7_and_final_merge_100m_x_768_nlist16384_nprobe64():
    """configs[3], second half: ranks 4-7 (and any the first test did not run), then the 8
    GPU records merged on the device (vdb_merge_ranks_packed_device, the merge every rank
    runs after the all-gather) against the oracle's merge of its 8 partials: the final
    cfg4 answer."""
    import torch
    c = CFG4
    for r in range(c["world"]):
        _cfg4_rank(r)
    e = _cfg4
    nq, k, world = c["nq"], c["k"], c["world"]
    with torch.cuda.stream(e["stream"]):
        od = torch.empty((nq, k), dtype=torch.float32, device=e["dev"])
        oi = torch.empty((nq, k), dtype=torch.int64, device=e["dev"])
        vdb.merge_ranks_packed_device(e["records"].data_ptr(), world, nq, k, od.data_ptr(), oi.data_ptr(),
                                      e["stream"].cuda_stream)
        torch.cuda.synchronize()
        D, I = od.cpu().numpy(), oi.cpu().numpy().view(np.uint64)
    Df, If = oracle.merge_ranks(e["oD"], e["oI"], k)
    sizes, scanned = e["sizes"], e["scanned"]
    _cfg4.clear()  # (releases the 100M-row assignment and the records)
    torch.cuda.empty_cache()
    assert np.array_equal(I, If), "final (merged) ids differ"
    assert np.array_equal(bits(D), bits(Df)), "final (merged) distance bits differ"
    assert int(sizes.sum()) == c["n"]
    assert sum(1 for x in scanned.values() if x) >= 2, "the probed lists should span several shards"
    # gpu_vs_cpu_test.cpp:209-219 validity rules on the final answer
    assert np.all(np.isfinite(D)) and np.all(D >= 0) and np.all(I < c["n"])
