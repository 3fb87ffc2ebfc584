#!/usr/bin/env python3
"""bench.py — QPS + p99 latency of MI355X IVF-Flat search (BASELINE.json metric).

Workload (BASELINE.json configs[2], the README headline): 10M x 768D fp32, nlist 4096,
nprobe 32, batch 64, k 10, L2. One step = one search of one batch of 64 queries
whose inputs are already in HBM. With N ranks (one per GPU, launched by
torch.distributed.run) every rank holds the lists the LPT shard plan gives it, scans
only those, and the per-rank top-k are all-gathered over RCCL and merged on device:
total work per batch is fixed, so scaling is "strong".

Index construction follows the reference benchmark (bench/benchmark.cpp:63-77):
train on the first 100K vectors (k-means++ from mt19937(42), 10 Lloyd iterations,
exactly ivf_flat_index.cpp:49-145), then add all vectors. Data are synthetic
iid N(0,1) draws generated on the device.

Rank 0 at N=1 also times the CPU oracle (oracle/, the restatement of the
reference's CPU search path) on a bounded sample of the same queries against the
same index, single-threaded like the reference (ivf_flat_index.cpp:214), and
checks the GPU results of that sample bit for bit.
"""
from __future__ import annotations

import argparse
import atexit
import ctypes
import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "cuda-acceleratedvectordatabaseengine_amd")

METRIC = "QPS + p99 latency, 10M×768D IVF-Flat k=10 nprobe=32, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def load_vdb():
    spec = importlib.util.spec_from_file_location("vdb_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vdb_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def percentile(values, p):
    """MetricsCollector::LatencyHistogram::percentile (server/query_service.cpp:790-798)."""
    s = sorted(values)
    return s[int(p * (len(s) - 1))] if s else 0.0


def mixture_centers(vdb, ncomp, group, dim, spread, device):
    """Two-level mixture: ncomp / group super-cluster centers S ~ N(0,1) (seed 777), and
    component j = S[j // group] + spread * N(0,1) (seed 778). Clustered data with locality:
    the group sibling components of a point's super-cluster are its nearest ones."""
    import torch
    s = torch.cuda.current_stream().cuda_stream
    nsup = (ncomp + group - 1) // group
    sup = torch.empty((nsup, dim), dtype=torch.float32, device=device)
    off = torch.empty((ncomp, dim), dtype=torch.float32, device=device)
    vdb.gen_normal_device(sup.data_ptr(), sup.numel(), seed=777, stream=s)
    vdb.gen_normal_device(off.data_ptr(), off.numel(), seed=778, stream=s)
    return sup.repeat_interleave(group, dim=0)[:ncomp] + spread * off


def fill_rows(vdb, args, buf, row0, m, seed, stream):
    """Rows row0 .. row0 + m of the synthetic stream `seed` into buf (device, m x dim):
    iid N(0,1) draws, or Gaussian-mixture draws around args.centers (--data mixture)."""
    if args.data == "mixture":
        vdb.gen_mixture_device(buf.data_ptr(), m, args.dim, args.centers.data_ptr(), args.centers.shape[0],
                               args.mix_sigma, seed, row0, stream)
    else:
        vdb.gen_normal_device(buf.data_ptr(), m * args.dim, seed=seed, offset=row0 * args.dim, stream=stream)


def build_index(vdb, args, device, rank, world):
    dim, n = args.dim, args.nvec
    stream = torch.cuda.current_stream().cuda_stream
    assert stream != 0, "run under an explicit torch stream (handle 0 means the engine's own stream)"
    data = torch.empty((n, dim), dtype=torch.float32, device=device)
    fill_rows(vdb, args, data, 0, n, 12345, stream)
    ids = torch.arange(n, dtype=torch.int64, device=device)
    torch.cuda.synchronize()
    idx = new_index(vdb, args, device)
    t0 = time.perf_counter()
    idx.train_device(data.data_ptr(), min(args.train, n))
    t1 = time.perf_counter()
    idx.add_device(data.data_ptr(), ids.data_ptr(), n)
    t2 = time.perf_counter()
    census(vdb, idx, args, data, min(args.train, n))
    del data, ids
    torch.cuda.empty_cache()
    log(rank, f"[bench] train {t1 - t0:.2f}s add {t2 - t1:.2f}s; index {idx.gpu_bytes_allocated() / 2**30:.1f} GiB on rank 0")
    return idx, {"train_s": round(t1 - t0, 3), "add_s": round(t2 - t1, 3)}


def new_index(vdb, args, device):
    # max_gpu_memory=0: every list HBM-resident (the reference's 8 GiB default Config cap
    # would put a 31 GB index on the list-cache tier)
    metric = vdb.Metric.InnerProduct if getattr(args, "metric", "l2") == "ip" else vdb.Metric.L2
    return vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(args.dim, args.nlist, metric, max_gpu_memory=0,
                                                    device=device.index))


def census(vdb, idx, args, rows, nrows):
    """--plan weighted: how many of the first --census rows of the database (query-like
    draws; the training sample) probe each list at the search's nprobe."""
    if getattr(args, "plan", "lpt") == "weighted" and getattr(args, "census_counts", None) is None:
        n = min(args.census, nrows)
        args.census_counts = (idx.probe_census(rows.data_ptr(), n, args.nprobe), n)


def shard_owners(vdb, args, sizes, world):
    """The shard plan: LPT on list sizes (default), or LPT on the expected scan cost per
    batch from the probe census (--plan weighted, vdb_shard_plan_probe_weighted)."""
    if getattr(args, "plan", "lpt") != "weighted":
        return None
    counts, n = args.census_counts
    return vdb.shard_plan_probe_weighted(sizes, counts, n, args.batch, world)


def sharded_assign(vdb, args, device, rank):
    """Pass 1 of the sharded build for an index larger than one GPU (configs[3]: 100M x 768
    = 307 GB): train on the first rows, then generate the database chunk by chunk (the
    same counter-based draws as one whole-array generation) and assign every row (exact
    argmin, assign_to_lists, ivf_flat_index.cpp:259-295) into a resident list-id array.
    Returns the trained (empty) index, the assignment and the final list sizes."""
    dim, n = args.dim, args.nvec
    stream = torch.cuda.current_stream().cuda_stream
    chunk = min(n, args.build_chunk)
    data = torch.empty((chunk, dim), dtype=torch.float32, device=device)
    asg = torch.empty(n, dtype=torch.int32, device=device)
    idx = new_index(vdb, args, device)
    t0 = time.perf_counter()
    ntrain = min(args.train, n)
    fill_rows(vdb, args, data, 0, ntrain, 12345, stream)
    torch.cuda.synchronize()
    idx.train_device(data.data_ptr(), ntrain)
    census(vdb, idx, args, data, ntrain)
    t1 = time.perf_counter()
    for a in range(0, n, chunk):
        m = min(chunk, n - a)
        fill_rows(vdb, args, data, a, m, 12345, stream)
        torch.cuda.synchronize()
        idx.assign_device(data.data_ptr(), m, asg[a:].data_ptr())
        log(rank, f"[bench] assigned {a + m} of {n} ({time.perf_counter() - t1:.1f}s)")
    sizes = torch.bincount(asg, minlength=args.nlist).cpu().numpy().astype(np.uint64)
    t2 = time.perf_counter()
    del data
    torch.cuda.empty_cache()
    return idx, asg, sizes, {"train_s": round(t1 - t0, 3), "assign_s": round(t2 - t1, 3)}


def sharded_append(vdb, args, device, idx, asg, sizes, rank, world):
    """Pass 2: the LPT plan from the final list sizes fixes this shard's lists (plan_shard),
    then every chunk is regenerated and only the owned lists' rows are appended. `world`
    is the number of shards (ranks, or --emulate-shard)."""
    dim, n = args.dim, args.nvec
    stream = torch.cuda.current_stream().cuda_stream
    chunk = min(n, args.build_chunk)
    data = torch.empty((chunk, dim), dtype=torch.float32, device=device)
    ids = torch.empty(chunk, dtype=torch.int64, device=device)
    t0 = time.perf_counter()
    idx.plan_shard(rank, world, sizes, owners=shard_owners(vdb, args, sizes, world))
    for a in range(0, n, chunk):
        m = min(chunk, n - a)
        fill_rows(vdb, args, data, a, m, 12345, stream)
        torch.arange(a, a + m, dtype=torch.int64, device=device, out=ids[:m])
        torch.cuda.synchronize()
        idx.add_to_lists_device(data.data_ptr(), ids.data_ptr(), asg[a:].data_ptr(), m)
    t1 = time.perf_counter()
    del data, ids
    torch.cuda.empty_cache()
    log(0, f"[bench] shard {rank}/{world}: append {t1 - t0:.2f}s, {idx.gpu_bytes_allocated() / 2**30:.1f} GiB, "
           f"largest list {int(sizes.max())}")
    return {"append_s": round(t1 - t0, 3), "sharded_build": f"shard {rank} of {world}"}


def build_index_sharded(vdb, args, device, rank, world):
    idx, asg, sizes, info = sharded_assign(vdb, args, device, rank)
    info.update(sharded_append(vdb, args, device, idx, asg, sizes, rank, world))
    del asg
    torch.cuda.empty_cache()
    return idx, info


def host_cpu_share():
    """Cores this process may use: the cgroup CPU quota (the GPU box gives one GPU's job a
    share of the host, while os.cpu_count() shows the whole machine), else os.cpu_count()."""
    n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def footprint(idx, args, world):
    """Device memory the index holds after the warm-up (the screen is built lazily by the
    first search): vdb_ivf_gpu_bytes_allocated (every list layout, centroids, workspaces)
    against the fp32 list bytes (count x dim x 4) and the reference's definition
    (get_gpu_memory_usage: count x (dim x 4 + 8) per resident list)."""
    sizes = idx.list_sizes()
    owned = idx.list_owners() if world > 1 or args.emulate_shard > 1 else None
    mine = sizes if owned is None else sizes[owned != 0xFFFFFFFF]
    fp32 = int(mine.sum()) * args.dim * 4
    alloc = idx.gpu_bytes_allocated()
    return {"gpu_bytes_allocated": alloc, "fp32_list_bytes": fp32,
            "over_fp32_lists": round(alloc / fp32, 3) if fp32 else None,
            "reference_gpu_memory_usage": idx.get_gpu_memory_usage()}


def timed_batch_parity(idx, args, queries, out_d, out_i):
    """The first TIMED batch's device results (one search call of B queries inside the timed
    region) against the oracle's search of the same B queries as one call (all cores)."""
    sys.path.insert(0, ROOT)
    import oracle  # test infrastructure: the checker only

    B, k = args.batch, args.k
    q0 = args.warmup * B
    qh = queries[q0:q0 + B].cpu().numpy()
    o = oracle.OracleIndex(args.dim, args.nlist, 0)
    o.centroids = idx.centroids
    sizes = idx.list_sizes()
    probed = set()
    for q in qh:
        probed.update(o.select_nprobe(q, args.nprobe).tolist())
    for l in sorted(probed):
        v, i = o.list_buffers(l, int(sizes[l]))
        if len(i):
            idx.get_list_into(l, v, i)
    t0 = time.perf_counter()
    D, I = o.search(qh, args.nprobe, k, threads=host_cpu_share())
    Dg, Ig = out_d[q0:q0 + B].cpu().numpy(), out_i[q0:q0 + B].cpu().numpy().view(np.uint64)
    same = bool(np.array_equal(I, Ig) and np.array_equal(D.view(np.uint32), Dg.view(np.uint32)))
    return {"batch": f"timed step 0 (queries {q0}..{q0 + B - 1}), one call", "bit_identical": same,
            "oracle_s": round(time.perf_counter() - t0, 1)}


def cpu_baseline(vdb, idx, args, queries_host, budget_s):
    """Time the oracle (reference CPU path restatement) on bounded query samples, the two
    numbers BASELINE.md promises: (1) one core, as the reference's serial query loop
    (ivf_flat_index.cpp:214), in calls of `--cpu-call` queries; (2) all cores this job may
    use (OpenMP over queries, bit-identical per query), one call of `--cpu-queries-mt`
    queries. The GPU answers the same calls (host API, untimed) and must match bit for bit;
    call boundaries matter (probe-slot reuse is per call, ivf_flat_index.cpp:210-211). The
    method follows gpu_vs_cpu_test.cpp:170-185: warm-up search, then the timed searches."""
    sys.path.insert(0, ROOT)
    import oracle  # test infrastructure: the CPU baseline leg only

    o = oracle.OracleIndex(args.dim, args.nlist, 0)
    o.centroids = idx.centroids
    n_mt = min(args.cpu_queries_mt, len(queries_host))
    sample = queries_host[: max(args.cpu_queries, n_mt)]
    probed = set()
    for q in sample:
        probed.update(o.select_nprobe(q, args.nprobe).tolist())
    sizes = idx.list_sizes()
    t_exp = time.perf_counter()
    for l in sorted(probed):  # only probed lists are ever read for these queries
        v, i = o.list_buffers(l, int(sizes[l]))
        if len(i):
            idx.get_list_into(l, v, i)
    t_exp = time.perf_counter() - t_exp
    o.search(sample[:2], args.nprobe, args.k)  # warm-up, as gpu_vs_cpu_test.cpp:171-172
    done, t_cpu = 0, 0.0
    parity = True
    single = sample[: args.cpu_queries]
    while done < len(single) and t_cpu < budget_s:
        chunk = single[done:done + args.cpu_call]
        t0 = time.perf_counter()
        D, I = o.search(chunk, args.nprobe, args.k, threads=1)
        t_cpu += time.perf_counter() - t0
        Dg, Ig = idx.search(chunk, nprobe=args.nprobe, k=args.k)
        parity &= bool(np.array_equal(I, Ig) and np.array_equal(D.view(np.uint32), Dg.view(np.uint32)))
        done += len(chunk)
    threads = host_cpu_share()
    mt = None
    if n_mt > 0:
        qs = sample[:n_mt]
        t0 = time.perf_counter()
        Dm, Im = o.search(qs, args.nprobe, args.k, threads=threads)
        t_mt = time.perf_counter() - t0
        Dg, Ig = idx.search(qs, nprobe=args.nprobe, k=args.k)
        parity_mt = bool(np.array_equal(Im, Ig) and np.array_equal(Dm.view(np.uint32), Dg.view(np.uint32)))
        mt = {"value": round(n_mt / t_mt, 3), "unit": "queries/s", "cores": threads,
              "sample": f"{n_mt} queries in one search() call, OpenMP over queries, {t_mt:.1f}s "
                        f"(bounded sample: BASELINE.md's Q = 1000 would take {1000 * t_mt / n_mt:.0f}s)",
              "parity_with_gpu": parity_mt}
        parity &= parity_mt
    return {
        "value": round(done / t_cpu, 3),
        "unit": "queries/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{done} queries of the timed workload (same index, nprobe {args.nprobe}, k {args.k}), "
                  f"oracle/cpu_ref.cpp single-threaded in calls of {args.cpu_call}, {t_cpu:.1f}s",
        "parity_with_gpu": parity,
        "all_cores": mt,
        "cpu_model": cpu_model(),
        "host_threads_visible": os.cpu_count(),
        "lists_exported_s": round(t_exp, 1),
    }


def host_api_leg(idx, args, queries, out_d, out_i):
    """The drop-in path a server uses: vdb_ivf_search from `--host-threads` caller
    threads, host buffers in and out (PCIe included), each call one batch of B queries
    (the rows of the timed steps), coalesced into device batches of at most
    `--host-coalesce` queries with up to three batches in flight. Checked bit for bit
    against the device-resident results of the same rows (same call boundaries)."""
    import threading
    B, k = args.batch, args.k
    q0 = args.warmup * B
    calls = [queries[q0 + j * B:q0 + (j + 1) * B].cpu().numpy() for j in range(args.steps)]
    ref_d = out_d[q0:q0 + args.steps * B].cpu().numpy()
    ref_i = out_i[q0:q0 + args.steps * B].cpu().numpy().view(np.uint64)
    idx.set_option("coalesce_max_queries", args.host_coalesce)
    for j in range(min(4, len(calls))):  # warm-up (staging buffers, streams)
        idx.search(calls[j], nprobe=args.nprobe, k=k)
    b0, r0 = idx.coalesce_stats()
    total = max(args.host_calls, len(calls))
    lock, nxt, same = threading.Lock(), [0], [True]

    def worker():
        while True:
            with lock:
                j = nxt[0]
                nxt[0] += 1
            if j >= total:
                return
            c = j % len(calls)
            D, I = idx.search(calls[c], nprobe=args.nprobe, k=k)
            if j < len(calls):
                ok = np.array_equal(I, ref_i[c * B:(c + 1) * B]) and \
                    np.array_equal(D.view(np.uint32), ref_d[c * B:(c + 1) * B].view(np.uint32))
                if not ok:
                    same[0] = False

    th = [threading.Thread(target=worker) for _ in range(args.host_threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    b1, r1 = idx.coalesce_stats()
    return {"value": round(total * B / el, 1), "unit": "queries/s", "calls": total, "queries_per_call": B,
            "caller_threads": args.host_threads, "device_batch_max_queries": args.host_coalesce,
            "device_batches": b1 - b0, "calls_per_device_batch": round((r1 - r0) / max(b1 - b0, 1), 2),
            "pcie_inclusive": True, "parity_with_device_path": same[0]}


def tier_leg(vdb, idx, args, device, queries):
    """configs[4]'s mechanism on one GPU: the index (or, for a sharded build, this rank's
    shard: a shard file with only its own lists' rows) is written to a file larger than
    the HBM list cache (vdb_ivf_save), a fresh handle serves it from that file through the
    list-cache tier (vdb_ivf_open_lists: io_uring reads, sub-batches cut to the cache,
    next sub-batch's lists loaded while the current one scans, next-use eviction), and
    calls of --tier-call queries are timed. Bytes read per batch of --batch queries are
    reported against the batch's algorithmic list bytes (the floor without a cache); the
    first call is checked bit for bit against the HBM-resident index it was saved from."""
    import tempfile
    d = args.tier_dir or tempfile.gettempdir()
    path = os.path.join(d, f"vdb_tier_{os.getpid()}.ivf")
    call = args.tier_call
    st = torch.cuda.current_stream()
    ref_d = torch.empty((call, args.k), dtype=torch.float32, device=device)
    ref_i = torch.empty((call, args.k), dtype=torch.int64, device=device)
    idx.search_device(queries.data_ptr(), call, args.nprobe, args.k, ref_d.data_ptr(), ref_i.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx.save(path)
    t_save = time.perf_counter() - t0
    file_bytes = os.path.getsize(path)
    shard_bytes = idx.get_gpu_memory_usage()  # this handle's lists, count * (dim * 4 + 8)
    cfg = vdb.IVFFlatIndex.Config(args.dim, args.nlist, vdb.Metric.L2, max_gpu_memory=0, device=device.index)
    idx.close()  # the HBM-resident index is gone: only the tier's cache holds lists now
    torch.cuda.empty_cache()
    try:
        h = vdb.IVFFlatIndex(cfg)
        h.set_option("list_cache_bytes", int(args.tier_cache_gib * (1 << 30)))
        h.set_option("batch", args.batch)
        h.open_lists(path)
        od = torch.empty((call, args.k), dtype=torch.float32, device=device)
        oi = torch.empty((call, args.k), dtype=torch.int64, device=device)
        calls = min(args.tier_calls, len(queries) // call)
        t0 = time.perf_counter()
        h.search_device(queries.data_ptr(), call, args.nprobe, args.k, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()  # (warm-up call: code objects, staging, the cache's first contents, the
        t_first = time.perf_counter() - t0  # screen's shadow built by streaming the file once)
        same = bool(torch.equal(oi, ref_i) and torch.equal(od.view(torch.int32), ref_d.view(torch.int32)))
        s0 = h.cache_stats()
        h.profile_enable(True)
        h.profile_reset()
        t0 = time.perf_counter()
        for j in range(1, calls):
            h.search_device(queries[j * call:].data_ptr(), call, args.nprobe, args.k, od.data_ptr(), oi.data_ptr(),
                            st.cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        prof = h.profile_read()
        s1 = h.cache_stats()
        nq = (calls - 1) * call
        batches = nq / args.batch
        alg = prof["scan_bytes"] / batches  # the lists each batch of --batch queries probes, read once
        read = (s1["file_bytes_read"] - s0["file_bytes_read"]) / batches
        screen = {}
        if s1["screen_resident"]:
            rows = s1["screen_rows_fetched"] - s0["screen_rows_fetched"]
            screen = {"screen": "the shadow, norms and ids of every stored list HBM-resident; the fp32 rows read "
                                "from the file only for the exact re-checks' survivors",
                      "screen_hbm_gb": round(s1["screen_bytes"] / 1e9, 2),
                      "survivor_rows_per_batch": round(rows / batches, 1),
                      "survivor_rows_from_hbm_cache_per_batch": round(
                          (s1.get("screen_rows_cached", 0) - s0.get("screen_rows_cached", 0)) / batches, 1),
                      "survivor_row_bytes_per_batch": int((s1["screen_row_bytes"] - s0["screen_row_bytes"]) / batches),
                      # file bytes read per byte of the survivor rows read (O_DIRECT granule supersets)
                      "read_amplification": round((s1["file_bytes_read"] - s0["file_bytes_read"]) /
                                                  max(s1["screen_row_bytes"] - s0["screen_row_bytes"], 1), 3),
                      "screen_batches": s1["screen_batches"] - s0["screen_batches"],
                      "screen_reruns": s1["screen_reruns"] - s0["screen_reruns"],
                      "first_call_s_incl_shadow_build": round(t_first, 1),
                      "collect_ms_per_batch": round(prof.get("collect_ms", 0.0) / max(prof["scan_launches"], 1), 3),
                      "search_ms_per_batch": round(prof["total_ms"] / max(prof["scan_launches"], 1), 3)}
        variants = []
        for vs in args.tier_variant:  # the same timed calls again under other engine options
            opts = [o.split("=") for o in vs.split(",") if o]
            for nm, v in opts:
                h.set_option(nm, int(v))
            v0 = h.cache_stats()
            t0 = time.perf_counter()
            for j in range(1, calls):
                h.search_device(queries[j * call:].data_ptr(), call, args.nprobe, args.k, od.data_ptr(), oi.data_ptr(),
                                st.cuda_stream)
            torch.cuda.synchronize()
            ev = time.perf_counter() - t0
            v1 = h.cache_stats()
            variants.append({"opts": vs, "value": round(nq / ev, 1),
                             "survivor_rows_from_hbm_cache_per_batch": round(
                                 (v1.get("screen_rows_cached", 0) - v0.get("screen_rows_cached", 0)) / batches, 1),
                             "survivor_rows_read_per_batch": round((v1["screen_rows_fetched"] - v0["screen_rows_fetched"]) / batches, 1),
                             "read_amplification": round((v1["file_bytes_read"] - v0["file_bytes_read"]) /
                                                         max(v1["screen_row_bytes"] - v0["screen_row_bytes"], 1), 3),
                             "file_read_gbps": round((v1["file_bytes_read"] - v0["file_bytes_read"]) / ev / 1e9, 2)})
            defaults = {"screen_recheck2": 1, "tier_row_direct": 1, "tier_row_cache": 1, "tier_row_qd": 256}
            for nm, v in opts:  # (back to the defaults for what follows)
                if nm in defaults:
                    h.set_option(nm, defaults[nm])
        if args.tier_adapt > 0 and s1["screen_resident"]:
            # the row cache refilled by the survivor rows that other queries (the queries'
            # generator, another seed: tier_adapt of them, served in calls) needed per list
            # (vdb_ivf_survivor_histogram: the rows per cached byte it would have saved), then
            # the same timed calls again
            aq = torch.empty((args.tier_adapt, args.dim), dtype=torch.float32, device=device)
            fill_rows(vdb, args, aq, 1 << 41, args.tier_adapt, 999, st.cuda_stream)
            h0 = h.survivor_histogram()
            for j in range(0, args.tier_adapt, call):
                n_ = min(call, args.tier_adapt - j)
                h.search_device(aq[j:].data_ptr(), n_, args.nprobe, args.k, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            del aq
            h.fill_row_cache(h.survivor_histogram() - h0)
            v0 = h.cache_stats()
            t0 = time.perf_counter()
            for j in range(1, calls):
                h.search_device(queries[j * call:].data_ptr(), call, args.nprobe, args.k, od.data_ptr(), oi.data_ptr(),
                                st.cuda_stream)
            torch.cuda.synchronize()
            ev = time.perf_counter() - t0
            v1 = h.cache_stats()
            variants.append({"opts": f"row cache by the survivor histogram of {args.tier_adapt} other queries", "value": round(nq / ev, 1),
                             "survivor_rows_from_hbm_cache_per_batch": round(
                                 (v1.get("screen_rows_cached", 0) - v0.get("screen_rows_cached", 0)) / batches, 1),
                             "survivor_rows_read_per_batch": round((v1["screen_rows_fetched"] - v0["screen_rows_fetched"]) / batches, 1),
                             "file_read_gbps": round((v1["file_bytes_read"] - v0["file_bytes_read"]) / ev / 1e9, 2)})
        if variants:
            screen["variants"] = variants
        return {"value": round(nq / el, 1), "unit": "queries/s", "calls": calls - 1, "queries_per_call": call, **screen,
                "file": path, "file_gb": round(file_bytes / 1e9, 2), "save_s": round(t_save, 1),
                "lists_gb": round(shard_bytes / 1e9, 2),
                "shard_file": args.emulate_shard > 1 or args.sharded_build,
                "cache_gib": args.tier_cache_gib, "cache_fraction_of_lists": round(args.tier_cache_gib * (1 << 30) / shard_bytes, 3),
                "file_bytes_read_per_batch": int(read), "algorithmic_bytes_per_batch": int(alg),
                "read_over_algorithmic": round(read / alg, 3) if alg else None,
                "file_read_gbps": round((s1["file_bytes_read"] - s0["file_bytes_read"]) / el / 1e9, 2),
                "subbatches": s1["subbatches"] - s0["subbatches"], "prefetches": s1["prefetches"] - s0["prefetches"],
                "sync_loads": s1["sync_loads"] - s0["sync_loads"], "io_uring": s1["io_uring"], "o_direct": s1["o_direct"],
                "batch": args.batch, "parity_with_resident_index": same}
    finally:
        os.unlink(path)


def shard_parity(vdb, idx, args, queries_host, rank, world):
    """Parity of one shard at full size: the oracle's shard search (oracle_search_shard:
    owned probed lists scanned, the others kept as counts for the empty-list rule,
    ivf_flat_index.cpp:225) against this handle's partial results for the same call. The
    shard is streamed into the checker one probed list at a time (exported from HBM,
    scanned for every query probing it, dropped), so its host memory is one list, not the
    shard."""
    sys.path.insert(0, ROOT)
    import oracle  # test infrastructure: the checker only

    o = oracle.OracleIndex(args.dim, args.nlist, 0)
    o.centroids = idx.centroids
    sample = queries_host[: args.shard_check]
    sizes = idx.list_sizes()
    owned = vdb.shard_plan(sizes, world) == rank
    t0 = time.perf_counter()
    D, I, loaded = o.search_shard_streamed(sample, args.nprobe, args.k, owned.astype(np.uint8), sizes,
                                           lambda l, v, i: idx.get_list_into(l, v, i), threads=16)
    t_cpu = time.perf_counter() - t0
    Dg, Ig = idx.search(sample, nprobe=args.nprobe, k=args.k)
    same = bool(np.array_equal(I, Ig) and np.array_equal(D.view(np.uint32), Dg.view(np.uint32)))
    return {"queries": len(sample), "shard": f"{rank} of {world}", "vectors_streamed": loaded,
            "oracle": "streamed, one list in host memory at a time, 16 threads", "oracle_s": round(t_cpu, 2),
            "bit_identical": same}


def lookup_traffic(path, key, build_id):
    """PMC HBM bytes per scan launch for workload `key`, measured by tools/pmc_traffic.py
    (rocprofv3 FETCH_SIZE, x2 gfx950 correction) ON A LIBRARY OF THIS BUILD ID: an entry
    taken on other kernel sources is stale, and the line then carries traffic null.
    Returns (bytes or None, a note saying which)."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, f"no traffic file ({os.path.basename(path)})"
    entry = tj.get("workloads", {}).get(key)
    if not entry:
        return None, f"no PMC entry for {key}"
    if entry.get("build_id") != build_id:
        return None, f"PMC entry for {key} was measured on build {entry.get('build_id')}, this library is {build_id}"
    return entry.get("hbm_bytes_per_scan_launch"), f"rocprofv3 FETCH_SIZE x2, build {build_id}"


def launch_ranks(n):
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--nvec", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--train", type=int, default=100_000)
    ap.add_argument("--cpu-queries", type=int, default=256, help="single-core CPU sample (bounded by --cpu-budget)")
    ap.add_argument("--cpu-queries-mt", type=int, default=128, help="all-cores CPU sample (one call)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--cpu-call", type=int, default=4, help="queries per oracle search() call")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check-batches", type=int, default=4,
                    help="N>1: timed batches checked bit-for-bit against the unsharded index")
    ap.add_argument("--exchange", default="engine", choices=["engine", "torch"],
                    help="N ranks: engine = the engine's own RCCL all-gather + merge inside vdb_ivf_search_device "
                         "(vdb_ivf_attach_comm); torch = the same packed records through torch.distributed")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="--exchange torch: nccl (RCCL) or gloo (host-staged rehearsal)")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (one-GPU rehearsal)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight (streams) in the timed region; 0 = 2 on one GPU (4: +5 %% QPS at "
                         "twice the p99), 3 across ranks (with the communicator's stream, 4 active hardware "
                         "queues: a fifth makes every queue slower, profiles/r05_sweep_slots.jsonl)")
    ap.add_argument("--latency-batches", type=int, default=1000,
                    help="batches per latency leg (p99 at the in-flight depth and one in flight; 0: p99 from the K steps)")
    ap.add_argument("--prof-steps", type=int, default=30,
                    help="single-stream steps timed per launch (roofline, one-in-flight latency)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per ivf_scan launch for this workload (or null)")
    ap.add_argument("--emulate-shard", type=int, default=0, metavar="W",
                    help="diagnostic: one process keeps one rank's LPT shard of W and runs its partial search "
                         "(the per-GPU work of a W-GPU node, without the all-gather); not a bench line")
    ap.add_argument("--emulate-rank", default="0", metavar="R",
                    help="with --emulate-shard: the rank emulated (0..W-1), or 'all' to time every rank's shard in "
                         "turn (sharded build) and report the per-rank balance")
    ap.add_argument("--plan", choices=["lpt", "weighted"], default="lpt",
                    help="shard plan: LPT on list sizes, or LPT on each list's expected scan cost per batch from a "
                         "probe census of --census training rows (vdb_shard_plan_probe_weighted)")
    ap.add_argument("--census", type=int, default=65536, help="rows of the probe census (--plan weighted)")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="N ranks, engine exchange: seconds before a communicator init or an exchange that has not "
                         "completed fails the run with an error naming the rank (option comm_timeout_ms)")
    ap.add_argument("--cfg", choices=["cfg2", "cfg3", "cfg4"], default=None,
                    help="BASELINE.json configs preset: cfg2 1M/256/16, cfg3 10M/4096/32 (default), "
                         "cfg4 100M/16384/64 (sharded build; on one GPU only with --emulate-shard 8)")
    ap.add_argument("--sharded-build", action="store_true",
                    help="assign pass, then each rank stores only its LPT lists (an index larger than one GPU)")
    ap.add_argument("--build-chunk", type=int, default=10_000_000, help="rows generated per build chunk")
    ap.add_argument("--shard-check", type=int, default=0, metavar="Q",
                    help="with --emulate-shard: check Q queries of this shard bit for bit against the oracle")
    ap.add_argument("--prewarm", action="store_true", help="warm every list up front (list-cache tier)")
    ap.add_argument("--data", choices=["iid", "mixture"], default="iid",
                    help="iid N(0,1) vectors (the reference generator's distribution; k-means makes hub lists), or a "
                         "Gaussian mixture (balanced lists, ~1.3 queries per probed list: the regime of clustered data)")
    ap.add_argument("--mix-components", type=int, default=0, help="mixture components (0 = nlist)")
    ap.add_argument("--mix-group", type=int, default=0,
                    help="components per super-cluster (0 = nprobe): a query's nprobe nearest lists are its siblings")
    ap.add_argument("--mix-spread", type=float, default=0.35, help="component centers around their super-cluster")
    ap.add_argument("--mix-sigma", type=float, default=0.1, help="points around their component center")
    ap.add_argument("--tier-cache-gib", type=float, default=0.0,
                    help="> 0: also serve the index from a file through the list-cache tier with this HBM cache")
    ap.add_argument("--tier-call", type=int, default=512, help="queries per search call in the tier leg")
    ap.add_argument("--tier-calls", type=int, default=8)
    ap.add_argument("--tier-variant", action="append", default=[], metavar="NAME=V[,NAME=V]",
                    help="tier leg: time the same calls again with these engine options (repeatable)")
    ap.add_argument("--tier-adapt", type=int, default=0, metavar="Q",
                    help="tier leg: also time the row cache refilled by the survivor histogram of Q other queries")
    ap.add_argument("--tier-dir", default="", help="directory for the tier leg's index file (default: TMPDIR)")
    ap.add_argument("--host-api", action="store_true",
                    help="also time the host API (vdb_ivf_search) from --host-threads caller threads")
    ap.add_argument("--host-threads", type=int, default=8)
    ap.add_argument("--host-calls", type=int, default=400, help="host-API calls of --batch queries each")
    ap.add_argument("--host-coalesce", type=int, default=64, help="max queries per coalesced device batch")
    ap.add_argument("--asg-file", default="", help=argparse.SUPPRESS)  # (a child of --emulate-rank all)
    ap.add_argument("--emulate-exchange", action="store_true",
                    help="--emulate-shard W: every batch also exchanges W records (world-1 all-gather) and merges them")
    ap.add_argument("--no-emulate-exchange", action="store_true",
                    help="--emulate-rank all: leave out the emulated all-gather + W-record merge per batch")
    ap.add_argument("--ranks-in-process", action="store_true",
                    help="--emulate-rank all in this one process (round 3's form) instead of a process per rank")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine tuning knob (vdb_ivf_set_option), e.g. wide_stride=1; results never change")
    args = ap.parse_args()
    if args.emulate_rank in ("all", "assign") or args.asg_file:
        args.sharded_build = True  # every rank's shard from one assignment pass
        args.emulate_shard = args.emulate_shard or 8
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # One process per GPU: launch the N ranks as children before anything touches
        # the GPU, wait for them, and exit with their status.
        sys.exit(launch_ranks(args.gpus))
    if args.cfg:
        args.nvec, args.nlist, args.nprobe = {"cfg2": (1_000_000, 256, 16), "cfg3": (10_000_000, 4096, 32),
                                              "cfg4": (100_000_000, 16384, 64)}[args.cfg]
        args.sharded_build |= args.cfg == "cfg4"
    if args.emulate_rank == "all" and not args.ranks_in_process:
        if args.inflight <= 0:
            args.inflight = 3
        sys.exit(run_emulated_ranks_procs(args))  # (before anything touches the GPU)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.inflight <= 0:
        # (3 batches in flight, one per workspace slot: round 6's two-pass re-check made the
        # third batch pay at one GPU too — cfg3 1.448 vs 1.513 ms per step at 2, same box,
        # profiles/r06_sweep_recheck2.jsonl; a batch's latency is then ~3 steps, p99 reported)
        args.inflight = 3
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()  # (does not initialise the GPU)
    if world > 1 and ndev < world:
        # fewer GPUs than ranks: a rehearsal of the N-rank protocol on the GPUs present,
        # with the exchange staged through host memory (RCCL wants one rank per GPU)
        args.same_device = True
    if world > 1 and args.same_device:  # RCCL wants one rank per GPU
        args.exchange, args.dist_backend = "torch", "gloo"
    args.rehearsal = world > 1 and args.same_device
    # control traffic (barriers, the timing max, the comm id) goes over gloo unless the
    # exchange itself is torch's nccl
    args.ctrl_dev = "cuda" if (args.exchange == "torch" and args.dist_backend == "nccl") else "cpu"
    device = torch.device("cuda", local_rank % max(ndev, 1) if args.same_device else local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        if args.ctrl_dev == "cuda":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    vdb = load_vdb()
    # Every kernel of this run (torch's and the engine's) goes to one explicit stream.
    with torch.cuda.stream(torch.cuda.Stream(device)):
        run(vdb, args, device, rank, world)
    if world > 1:
        dist.destroy_process_group()


def device_wait(args, world, idx, streams, rank):
    """Wait for `streams` (torch.cuda.synchronize semantics). With the engine's own
    communicator a stalled peer must not hang the run: the engine's watchdog marks an
    exchange that misses comm_timeout_ms failed, and this rank then prints the error naming
    itself and exits non-zero (the driver's launcher tears the other ranks down)."""
    if world == 1 or args.exchange != "engine" or idx is None:
        torch.cuda.synchronize()
        return
    evs = []
    for st in streams:
        e = torch.cuda.Event()
        e.record(st)
        evs.append(e)
    while not all(e.query() for e in evs):
        err, issued, done = idx.comm_status()
        if err:
            print(json.dumps({"error": err, "rank": rank, "exchanges_issued": issued, "exchanges_done": done}),
                  flush=True)
            print(f"[bench] rank {rank}: {err}", file=sys.stderr, flush=True)
            os._exit(3)  # (no teardown: the stalled collective is still queued on the device)
        time.sleep(0.001)
    torch.cuda.synchronize()


def attach_engine_comm(vdb, idx, args, rank, world):
    """The engine's own communicator: rank 0 draws the RCCL id, the others receive it over
    the control group; init is non-blocking with a deadline (option comm_timeout_ms)."""
    idx.set_option("comm_timeout_ms", int(args.comm_timeout * 1000))
    cid = torch.zeros(vdb.COMM_ID_BYTES, dtype=torch.uint8)
    if rank == 0:
        cid.copy_(torch.frombuffer(bytearray(vdb.comm_unique_id()), dtype=torch.uint8))
    dist.broadcast(cid, src=0)
    try:
        idx.attach_comm(bytes(cid.numpy().tobytes()), rank, world)
    except Exception as e:  # noqa: BLE001 — report which rank failed, exit non-zero
        print(json.dumps({"error": str(e), "rank": rank}), flush=True)
        print(f"[bench] rank {rank}: attach_comm failed: {e}", file=sys.stderr, flush=True)
        os._exit(3)


_DEDICATED_STREAMS = []


def dedicated_streams(device, n):
    """n streams, each on a hardware queue of its own. A plain stream takes the least-used of
    the process's 4 queues when it is first used, so two of three batches in flight could
    share a queue with a stream used earlier (the build's) and serialise: the 1/8 shard's step
    at 3 in flight was 0.29 or 0.40 ms depending on which streams a run picked
    (profiles/r05_hw_queue_probe.txt). A stream with a CU mask gets a queue of its own; the
    mask enables every CU. (Falls back to plain streams if the call is unavailable.)"""
    try:
        path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
        hip = ctypes.CDLL(path)
        ncu = torch.cuda.get_device_properties(device).multi_processor_count
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
        out = []
        for _ in range(n):
            h = ctypes.c_void_p()
            if hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask) != 0:
                raise RuntimeError("hipExtStreamCreateWithCUMask failed")
            if not _DEDICATED_STREAMS:
                atexit.register(_destroy_dedicated_streams)
            _DEDICATED_STREAMS.append((hip, h))
            out.append(torch.cuda.ExternalStream(h.value, device=device))
        return out
    except Exception:
        return [torch.cuda.Stream(device) for _ in range(n)]


def _destroy_dedicated_streams():
    if _DEDICATED_STREAMS:
        torch.cuda.synchronize()
    while _DEDICATED_STREAMS:
        hip, h = _DEDICATED_STREAMS.pop()
        hip.hipStreamDestroy(h)


def timed_region(vdb, idx, args, device, rank, world, queries, out_d, out_i, check=None):
    """W warm-up steps, then exactly K timed steps with `inflight` batches in flight,
    bracketed by barrier + synchronize, max over ranks; then the roofline pass: the same
    steps one at a time on one stream, so the engine's per-batch events time each scan
    launch on its own (and give the latency of a batch with nothing else in flight)."""
    B, k = args.batch, args.k
    # Batches in flight: step s runs on streams[s % inflight]; the engine gives each
    # concurrent search its own workspace slot, so one batch's small kernels and scan
    # tail overlap the next batch's scan. Rank partials and gathers are per stream. Each
    # stream has a hardware queue of its own (dedicated_streams).
    torch.cuda.synchronize()
    streams = dedicated_streams(device, args.inflight)
    # One packed record per rank and batch (f32 dist[B][k] | pad | u64 ids[B][k]): ONE
    # all-gather per batch over RCCL, then the on-device merge of the world records.
    rec = vdb.rank_record_bytes(B, k)
    ids_off = vdb.rank_record_ids_offset(B, k)
    part = [torch.empty(rec, dtype=torch.uint8, device=device) for _ in streams]
    gat = [torch.empty(world * rec, dtype=torch.uint8, device=device) for _ in streams]
    torch.cuda.synchronize()
    ctrl = device if args.ctrl_dev == "cuda" else "cpu"

    def step(s, slot):
        st = streams[slot]
        q = queries[s * B:(s + 1) * B]
        with torch.cuda.stream(st):
            if world == 1 or args.exchange == "engine":  # (engine exchange: final results on every rank)
                idx.search_device(q.data_ptr(), B, args.nprobe, k, out_d[s * B:].data_ptr(), out_i[s * B:].data_ptr(),
                                  st.cuda_stream)
            else:
                p0 = part[slot].data_ptr()
                idx.search_device(q.data_ptr(), B, args.nprobe, k, p0, p0 + ids_off, st.cuda_stream)
                if args.dist_backend == "nccl":
                    dist.all_gather_into_tensor(gat[slot], part[slot])
                else:  # gloo (one-GPU rehearsal): the same exchange staged through host memory
                    h = torch.empty(world * rec, dtype=torch.uint8)
                    dist.all_gather_into_tensor(h, part[slot].cpu())
                    gat[slot].copy_(h)
                vdb.merge_ranks_packed_device(gat[slot].data_ptr(), world, B, k, out_d[s * B:].data_ptr(),
                                              out_i[s * B:].data_ptr(), st.cuda_stream)

    for s in range(args.warmup):
        step(s, s % len(streams))
    device_wait(args, world, idx, streams, rank)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.steps):
        slot = j % len(streams)
        starts[j].record(streams[slot])
        step(args.warmup + j, slot)
        ends[j].record(streams[slot])
    device_wait(args, world, idx, streams, rank)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    parity_multi = None
    if check is not None:
        q0, nchk, chk_d, chk_i = check
        same = bool(torch.equal(out_i[q0:q0 + nchk], chk_i) and
                    torch.equal(out_d[q0:q0 + nchk].view(torch.int32), chk_d.view(torch.int32)))
        flag = torch.tensor([1 if same else 0], dtype=torch.int32, device=ctrl)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        parity_multi = bool(int(flag.item()) == 1)
    lat = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    p99_steps = percentile(lat, 0.99)
    if world > 1:
        t = torch.tensor([elapsed, p99_steps], dtype=torch.float64, device=ctrl)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, p99_steps = float(t[0]), float(t[1])
    # p99 latency from its own leg (QPS stays the K timed steps'): with K = 20 a "p99" is the
    # second-largest sample, so the latency legs time >= 1000 batches each, at the same
    # in-flight depth (closed loop: batch j is issued when batch j - depth completes, so its
    # start event fires at issue) and one at a time
    lat_legs = {}
    if args.latency_batches > 0:
        for depth in sorted({len(streams), 1}, reverse=True):
            lat_legs[depth] = latency_leg(args, world, idx, rank, streams[:depth], step, ctrl)
    if lat_legs:
        p99, lat_mean = lat_legs[len(streams)]["p99_ms"], lat_legs[len(streams)]["mean_ms"]
    else:
        p99, lat_mean = p99_steps, sum(lat) / max(len(lat), 1)

    device_wait(args, world, idx, streams, rank)
    idx.profile_enable(True)
    idx.set_option("bounded_stats", 1)  # the screen's re-check count (roofline bytes); never changes results
    idx.profile_reset()
    s_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.prof_steps)]
    e_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.prof_steps)]
    for j in range(args.prof_steps):
        s_ev[j].record(streams[0])
        step(args.warmup + args.steps + j, 0)
        e_ev[j].record(streams[0])
    device_wait(args, world, idx, streams, rank)
    prof = idx.profile_read()
    idx.profile_enable(False)
    idx.set_option("bounded_stats", 0)
    step_ms_single = [a.elapsed_time(b) for a, b in zip(s_ev, e_ev)]
    p99_single = percentile(step_ms_single, 0.99)
    mine = rank_breakdown(rank, prof, elapsed * 1e3 / max(args.steps, 1), step_ms_single)
    if args.rehearsal:
        # The ranks of a rehearsal share one GPU: a phase's HIP-event interval on one rank also
        # holds the other ranks' kernels that run meanwhile. The same local searches once more,
        # the ranks taking turns (a barrier between them, nothing else on the GPU), give each
        # rank's own phase times.
        idx.profile_enable(True)
        idx.profile_reset()
        st = streams[0]
        for j in range(args.prof_steps):
            q = queries[(args.warmup + args.steps + j) * B:]
            for r in range(world):
                dist.barrier()
                if r == rank:
                    idx.search_device(q.data_ptr(), B, args.nprobe, k, part[0].data_ptr(), part[0].data_ptr() + ids_off,
                                      st.cuda_stream)
                    st.synchronize()
        dist.barrier()
        pa = idx.profile_read()
        idx.profile_enable(False)
        na = max(pa["scan_launches"], 1)
        mine["ranks_taking_turns"] = {"scan_ms": round(pa["scan_ms"] / na, 4), "coarse_ms": round(pa["coarse_ms"] / na, 4),
                                      "local_merge_ms": round(pa.get("local_merge_ms", 0.0) / na, 4),
                                      "search_ms": round(pa["total_ms"] / na, 4)}
    per_rank = None
    if world > 1:
        t = torch.tensor([p99_single], dtype=torch.float64, device=ctrl)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        p99_single = float(t[0])
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    if 1 in lat_legs:
        p99_single = lat_legs[1]["p99_ms"]
    return {"elapsed": elapsed, "p99": p99, "lat_mean": lat_mean, "p99_single": p99_single, "prof": prof,
            "p99_steps": p99_steps, "latency_legs": lat_legs,
            "parity_multi": parity_multi,
            "per_rank": per_rank, "mine": mine}


def latency_leg(args, world, idx, rank, streams, step, ctrl):
    """args.latency_batches batches at len(streams) in flight, closed loop: batch j is issued
    (on streams[j % depth]) once batch j - depth has completed, so its start event fires at
    issue and its latency is issue -> results ready (device time, including the other
    batches in flight). Queries cycle over the bench's query set; every batch writes the
    same results to the same output rows as its first use. p99 = sorted[floor(0.99 (n-1))]
    (query_service.cpp:790-798), max over ranks."""
    depth, n = len(streams), args.latency_batches
    nq_batches = args.warmup + args.steps + args.prof_steps
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n)]

    def wait(e):
        while not e.query():
            if world > 1 and args.exchange == "engine":
                err = idx.comm_status()[0]
                if err:
                    print(json.dumps({"error": err, "rank": rank}), flush=True)
                    os._exit(3)
            time.sleep(0.00002)

    device_wait(args, world, idx, streams, rank)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for j in range(n):
        if j >= depth:
            wait(ends[j - depth])
        st = streams[j % depth]
        starts[j].record(st)
        step(j % nq_batches, j % depth)
        ends[j].record(st)
    device_wait(args, world, idx, streams, rank)
    wall = time.perf_counter() - t0
    lat = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    out = [percentile(lat, 0.99), sum(lat) / n, percentile(lat, 0.5), max(lat), wall]
    if world > 1:
        t = torch.tensor(out, dtype=torch.float64, device=ctrl)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out = [float(x) for x in t]
    return {"inflight": depth, "samples": n, "p99_ms": round(out[0], 4), "mean_ms": round(out[1], 4),
            "p50_ms": round(out[2], 4), "max_ms": round(out[3], 4), "qps": round(n * args.batch / out[4], 1)}


def rank_breakdown(rank, prof, ms_per_step, step_ms_single):
    """One rank's per-batch phases from the engine's HIP events (roofline pass, one batch
    in flight): scan, the merges after it, and at N>1 the exchange (this rank's record
    ready -> all-gather done: the wait for the slowest rank plus the collective) and the
    rank merge."""
    n = max(prof["scan_launches"], 1)
    x = max(prof.get("exchanges", 0), 1)
    return {"rank": rank, "scan_ms": round(prof["scan_ms"] / n, 4),
            "coarse_ms": round(prof["coarse_ms"] / n, 4),
            "local_merge_ms": round(prof.get("local_merge_ms", 0.0) / n, 4),
            "search_ms": round(prof["total_ms"] / n, 4),
            "exchange_wait_ms": round(prof.get("exchange_ms", 0.0) / x, 4) if prof.get("exchanges") else None,
            "rank_merge_ms": round(prof.get("rank_merge_ms", 0.0) / x, 4) if prof.get("exchanges") else None,
            "step_ms_one_in_flight": round(sum(step_ms_single) / max(len(step_ms_single), 1), 4),
            "ms_per_step": round(ms_per_step, 4),
            "scan_bytes_per_batch": int(prof["scan_bytes"] / max(prof["batches"], 1)),
            "distances_per_batch": int(prof["pair_vectors"] / max(prof["batches"], 1)),
            "distinct_lists_per_batch": round(prof["distinct_lists"] / max(prof["batches"], 1), 1)}


def balance(per_rank):
    """max / min over ranks of the per-rank phases (1.0 = perfectly balanced shards)."""
    out = {}
    for key in ("scan_ms", "search_ms", "ms_per_step", "scan_bytes_per_batch", "distances_per_batch"):
        v = [r[key] for r in per_rank if r and r.get(key)]
        if v:
            out[key] = {"max": max(v), "min": min(v), "max_over_min": round(max(v) / min(v), 4),
                        "argmax_rank": per_rank[[r[key] if r else None for r in per_rank].index(max(v))]["rank"]}
    return out


def make_queries(vdb, args, device):
    B, k = args.batch, args.k
    nq = (args.warmup + args.steps + args.prof_steps) * B
    queries = torch.empty((nq, args.dim), dtype=torch.float32, device=device)
    fill_rows(vdb, args, queries, 0, nq, 12346, torch.cuda.current_stream().cuda_stream)
    out_d = torch.empty((nq, k), dtype=torch.float32, device=device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=device)
    return queries, out_d, out_i


def child_argv(rank_arg, asg_file):
    """This command line with --emulate-rank replaced (a child of the emulated-ranks run)."""
    out, skip = [], False
    for a in sys.argv[1:]:
        if skip:
            skip = False
            continue
        if a == "--emulate-rank":
            skip = True
            continue
        if a.startswith("--emulate-rank="):
            continue
        out.append(a)
    return [sys.executable, "-u", os.path.abspath(__file__)] + out + ["--emulate-rank", rank_arg, "--asg-file", asg_file]


def child_argv_inflight(args, rank_arg, asg_file):
    return child_argv(rank_arg, asg_file) + ["--inflight", str(args.inflight)]


def run_emulated_ranks_procs(args):
    """--emulate-rank all: every rank of a W-GPU node in a process of its own, one after
    the other on this one GPU, as on a real node (one process per GPU): a first child runs
    the assignment pass and writes the centroids, the assignment and the list sizes to a
    file; child r builds rank r's LPT shard from it and times it. A fresh process per rank
    keeps one rank's streams, allocations and code objects from shaping the next rank's
    timing (round 3 timed the ranks in one process: even ranks stepped 1.4x slower than
    odd ones at equal scan times). The parent never touches the GPU."""
    import subprocess
    import tempfile
    W = args.emulate_shard
    f = os.path.join(args.tier_dir or tempfile.gettempdir(), f"vdb_asg_{os.getpid()}.npz")
    ranks, info = [], {}
    try:
        r = subprocess.run(child_argv_inflight(args, "assign", f), stdout=subprocess.PIPE, text=True)
        sys.stdout.write("".join(l + "\n" for l in r.stdout.splitlines() if not l.startswith("ASSIGN ")))
        if r.returncode != 0:
            return r.returncode
        info = json.loads([l for l in r.stdout.splitlines() if l.startswith("ASSIGN ")][-1][7:])
        for rk in range(W):
            r = subprocess.run(child_argv_inflight(args, str(rk), f), stdout=subprocess.PIPE, text=True)
            rows = [l for l in r.stdout.splitlines() if l.startswith("RANKROW ")]
            if r.returncode != 0 or not rows:
                sys.stdout.write(r.stdout)
                return r.returncode or 1
            ranks.append(json.loads(rows[-1][8:]))
            log(0, f"[bench] emulated rank {rk}/{W}: " + rows[-1][8:])
        with np.load(f) as z:
            sizes = z["sizes"]
    finally:
        if os.path.exists(f):
            os.unlink(f)
    plan = vdb_plan_host(args, sizes, W)
    lists = [int((plan == r).sum()) for r in range(W)]
    vecs = [int(sizes[plan == r].sum()) for r in range(W)]
    print(json.dumps({
        "metric": f"per-rank balance of the {W}-GPU LPT shard plan (emulated on one GPU)",
        "unit": "ms", "n_gpus": 1, "emulated_ranks": W, "steps": args.steps, "warmup": args.warmup,
        "config": {"workload": f"{args.nvec // 1_000_000}M x {args.dim}D IVF-Flat L2, nlist {args.nlist}, "
                               f"nprobe {args.nprobe}, batch {args.batch}, k {args.k}",
                   "inflight": args.inflight, "data": args.data},
        "plan": args.plan, "ranks": ranks, "balance": balance(ranks),
        "shard_lists": lists, "shard_vectors": vecs,
        "predicted_8gpu_qps_from_max_rank_step": round(args.batch * 1e3 / max(r["ms_per_step"] for r in ranks), 1),
        "build": info, "process_per_rank": True,
        "exchange": ("excluded" if args.no_emulate_exchange else
                     f"on every batch: an RCCL all-gather of {W} records' bytes (communicator of world 1: a "
                     f"local copy, not the xGMI latency) and the on-device merge of {W} records"),
        "note": "per-rank results; each rank's search timed alone, in its own process",
    }), flush=True)
    return 0


def vdb_plan_host(args, sizes, W):
    """The LPT owner of every list (host only; no GPU)."""
    vdb = load_vdb()
    return vdb.shard_plan(sizes, W)


def emulated_assign(vdb, args, device):
    """The assignment child of --emulate-rank all: pass 1 of the sharded build, saved."""
    trained, asg, sizes, info = sharded_assign(vdb, args, device, 0)
    np.savez(args.asg_file, centroids=trained.centroids, asg=asg.cpu().numpy(), sizes=sizes)
    trained.close()
    print("ASSIGN " + json.dumps(info), flush=True)


def emulated_rank(vdb, args, device, r):
    """Rank r's child of --emulate-rank all: its LPT shard from the saved assignment, timed."""
    W = args.emulate_shard
    with np.load(args.asg_file) as z:
        centroids, asg, sizes = z["centroids"], torch.from_numpy(z["asg"]).to(device), z["sizes"]
    queries, out_d, out_i = make_queries(vdb, args, device)
    idx = new_index(vdb, args, device)
    idx.centroids = centroids
    binfo = sharded_append(vdb, args, device, idx, asg, sizes, r, W)
    del asg
    torch.cuda.empty_cache()
    for o in args.opt:
        name, val = o.split("=", 1)
        idx.set_option(name, int(val))
    if not args.no_emulate_exchange:
        # every batch also carries what a W-GPU node adds per rank: the all-gather (an RCCL
        # communicator of world 1 gathering W records' bytes) and the W-record rank merge
        idx.set_option("exchange_emulate_world", W)
        idx.attach_comm(vdb.comm_unique_id(), 0, 1)
    res = timed_region(vdb, idx, args, device, 0, 1, queries, out_d, out_i)
    row = dict(res["mine"], rank=r, qps=round(args.steps * args.batch / res["elapsed"], 1),
               p99_ms=round(res["p99"], 4), latency_mean_ms=round(res["lat_mean"], 4),
               p99_ms_one_in_flight=round(res["p99_single"], 4),
               shard_gib=round(idx.gpu_bytes_allocated() / 2**30, 2), append_s=binfo["append_s"])
    print("RANKROW " + json.dumps(row), flush=True)


def run_emulated_ranks(vdb, args, device):
    """--emulate-rank all: the per-GPU work of every rank of a W-GPU node, timed in turn on
    this one GPU. One sharded-build assignment pass; then for each rank r a fresh index
    holding exactly rank r's LPT lists (plan_shard + append), the same K timed steps of its
    partial search, and its per-batch phases; the line reports every rank and the
    max/min balance (the 8-GPU step is the max over ranks). Partial results only: a
    diagnostic line, not the bench line."""
    W = args.emulate_shard
    trained, asg, sizes, info = sharded_assign(vdb, args, device, 0)
    centroids = trained.centroids
    trained.close()
    queries, out_d, out_i = make_queries(vdb, args, device)
    ranks = []
    for r in range(W):
        idx = new_index(vdb, args, device)
        idx.centroids = centroids
        binfo = sharded_append(vdb, args, device, idx, asg, sizes, r, W)
        for o in args.opt:
            name, val = o.split("=", 1)
            idx.set_option(name, int(val))
        res = timed_region(vdb, idx, args, device, 0, 1, queries, out_d, out_i)
        row = dict(res["mine"], rank=r, qps=round(args.steps * args.batch / res["elapsed"], 1),
                   p99_ms=round(res["p99"], 4), latency_mean_ms=round(res["lat_mean"], 4),
                   p99_ms_one_in_flight=round(res["p99_single"], 4),
                   shard_gib=round(idx.gpu_bytes_allocated() / 2**30, 2), append_s=binfo["append_s"])
        log(0, f"[bench] emulated rank {r}/{W}: " + json.dumps(row))
        ranks.append(row)
        idx.close()
        torch.cuda.empty_cache()
    plan = shard_owners(vdb, args, sizes, W)
    if plan is None:
        plan = vdb.shard_plan(sizes, W)
    lists = [int((plan == r).sum()) for r in range(W)]
    vecs = [int(sizes[plan == r].sum()) for r in range(W)]
    return {
        "metric": f"per-rank balance of the {W}-GPU LPT shard plan (emulated on one GPU)",
        "unit": "ms", "n_gpus": 1, "emulated_ranks": W, "steps": args.steps, "warmup": args.warmup,
        "config": {"workload": f"{args.nvec // 1_000_000}M x {args.dim}D IVF-Flat L2, nlist {args.nlist}, "
                               f"nprobe {args.nprobe}, batch {args.batch}, k {args.k}",
                   "inflight": args.inflight, "data": args.data},
        "plan": args.plan, "ranks": ranks, "balance": balance(ranks),
        "shard_lists": lists, "shard_vectors": vecs,
        "predicted_8gpu_qps_from_max_rank_step": round(args.batch * 1e3 / max(r["ms_per_step"] for r in ranks), 1),
        "build": info, "note": "partial (per-rank) results; exchange excluded; each rank's search timed alone",
    }


def run(vdb, args, device, rank, world):
    if args.data == "mixture":
        args.centers = mixture_centers(vdb, args.mix_components or args.nlist, args.mix_group or args.nprobe,
                                       args.dim, args.mix_spread, device)
    if args.emulate_rank == "all":  # (--ranks-in-process: the round-3 form, every rank in this process)
        line = run_emulated_ranks(vdb, args, device)
        print(json.dumps(line), flush=True)
        return
    if args.emulate_rank == "assign":
        emulated_assign(vdb, args, device)
        return
    if args.asg_file:
        emulated_rank(vdb, args, device, int(args.emulate_rank))
        return
    er = int(args.emulate_rank)
    if args.sharded_build:
        shards = world if world > 1 else max(args.emulate_shard, 1)
        idx, build_info = build_index_sharded(vdb, args, device, rank if world > 1 else er, shards)
    else:
        idx, build_info = build_index(vdb, args, device, rank, world)
    for o in args.opt:
        name, val = o.split("=", 1)
        idx.set_option(name, int(val))
    if args.prewarm:  # list-cache tier: load every list up front, in list order (vdb.QueryService/Warmup)
        idx.warmup_lists(list(range(args.nlist)))
    if args.emulate_shard > 1 and world == 1 and not args.sharded_build:
        idx.set_shard(er, args.emulate_shard, owners=shard_owners(vdb, args, idx.list_sizes(), args.emulate_shard))
    B, k = args.batch, args.k
    queries, out_d, out_i = make_queries(vdb, args, device)
    main_stream = torch.cuda.current_stream()
    check = None
    if world > 1 and not args.sharded_build:
        # Reference for the end-to-end check: the whole (unsharded) index answers the
        # first timed batches on this rank before it keeps only its LPT shard.
        nchk = min(args.check_batches, args.steps) * B
        q0 = args.warmup * B
        chk_d = torch.empty((nchk, k), dtype=torch.float32, device=device)
        chk_i = torch.empty((nchk, k), dtype=torch.int64, device=device)
        for b0 in range(0, nchk, B):
            idx.search_device(queries[q0 + b0:].data_ptr(), B, args.nprobe, k, chk_d[b0:].data_ptr(),
                              chk_i[b0:].data_ptr(), main_stream.cuda_stream)
        torch.cuda.synchronize()
        check = (q0, nchk, chk_d, chk_i)
        idx.set_shard(rank, world, owners=shard_owners(vdb, args, idx.list_sizes(), world))
    if world > 1 and args.exchange == "engine":
        attach_engine_comm(vdb, idx, args, rank, world)
    if world == 1 and args.emulate_shard > 1 and args.emulate_exchange:
        # (this rank's timeline with the per-batch exchange of a W-GPU node: an all-gather of W
        # records' bytes on a communicator of world 1 and the W-record merge)
        idx.set_option("exchange_emulate_world", args.emulate_shard)
        idx.attach_comm(vdb.comm_unique_id(), 0, 1)
    res = timed_region(vdb, idx, args, device, rank, world, queries, out_d, out_i, check)
    elapsed, p99, p99_single, prof = res["elapsed"], res["p99"], res["p99_single"], res["prof"]
    parity_multi = res["parity_multi"]

    launches = max(prof["scan_launches"], 1)
    scan_ms = prof["scan_ms"] / launches
    batches = max(prof["batches"], 1)
    fp32_bytes = prof["scan_bytes"] / batches  # 4 D per vector of the batch's distinct probed lists
    # The screened scan (default) streams the lists' bf16 residual shadow (2 dp B per vector)
    # and 16 B of norms, and reads the fp32 row (4 dp B) of every re-checked pair: its
    # algorithmic bytes. The exact scan reads the fp32 lists once per batch.
    screened = prof.get("bounded_blocks", 0) > 0
    deferred = screened and prof.get("collect_ms", 0) > 0
    dp = -(-args.dim // 64) * 64
    collect_ms = prof.get("collect_ms", 0.0) / launches
    # the deferred screen's shadow: bf16, or int8 + a 4 B scale per vector (option screen_i8: the
    # engine chooses by default, profile field screen_shadow says which it built)
    shadow_i8 = deferred and prof.get("screen_shadow", 1) == 2
    shadow_b = dp + 4 if shadow_i8 else 2 * dp
    if deferred:
        # the dominant kernel is the deferred screen's collect pass: it streams the shadow and
        # the norms and writes 16 B per collected (query, vector) pair; the exact re-checks
        # after it read 4 dp B per survivor (reported beside it)
        vecs = prof["scan_vectors"] / batches
        collected = prof.get("screen_collected", 0) / batches
        bytes_per_launch = vecs * (shadow_b + 16) + collected * 16
        kernel_ms = collect_ms
    elif screened:
        vecs = prof["scan_vectors"] / batches
        rechecks = prof["exact_reranks"] / batches
        bytes_per_launch = vecs * (2 * dp + 16) + rechecks * 4 * dp
        kernel_ms = scan_ms
    else:
        bytes_per_launch = fp32_bytes
        kernel_ms = scan_ms
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    key = f"{args.nvec}x{args.dim}/{args.nlist}/{args.nprobe}/{B}/{k}/N{world}"
    if args.data != "iid":
        key += f"/{args.data}"
    if args.emulate_shard > 1:
        key += f"/shard{er}of{args.emulate_shard}"
    if args.opt:  # knobs can change the traffic (never the results)
        key += "/" + ",".join(sorted(args.opt))
    traffic, traffic_note = lookup_traffic(args.traffic_json, key, vdb.build_id())

    result = {
        "metric": METRIC,
        "value": round(args.steps * B / elapsed, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "p99_ms": round(p99, 4),
        "p99_ms_one_in_flight": round(p99_single, 4),
        # (p99 from >= 1000-batch latency legs; the K timed steps' own p99 beside it)
        "p99_samples": args.latency_batches if res["latency_legs"] else args.steps,
        "p99_ms_timed_steps": round(res["p99_steps"], 4),
        "latency_legs": list(res["latency_legs"].values()),
        # with `inflight` batches in flight a batch's latency is at least inflight x ms_per_step
        # on average (Little's law); p99 / mean shows the spread around that
        "latency_mean_ms": round(res["lat_mean"], 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic: iid N(0,1) fp32 vectors generated on device (seed 12345), queries seed 12346"
                 if args.data == "iid" else
                 f"synthetic: two-level Gaussian mixture, {args.centers.shape[0]} components in super-clusters of "
                 f"{args.mix_group or args.nprobe} (supers N(0,1) seed 777, components +{args.mix_spread} N(0,1) seed 778, "
                 f"points +{args.mix_sigma} N(0,1)) generated on device (seed 12345), queries from the same mixture "
                 f"(seed 12346)"),
        "config": {
            "workload": f"{args.nvec // 1_000_000}M x {args.dim}D IVF-Flat L2, nlist {args.nlist}, nprobe {args.nprobe}, "
                        f"batch {B}, k {k}",
            "nvec": args.nvec, "dim": args.dim, "nlist": args.nlist, "nprobe": args.nprobe, "batch": B, "k": k,
            "train_vectors": min(args.train, args.nvec),
            "parallelism": (f"lists sharded over {world} rank(s) ({'probe-weighted ' if args.plan == 'weighted' else ''}LPT), one all-gather per batch of per-rank top-k "
                            + (" (engine RCCL communicator, vdb_ivf_attach_comm)" if args.exchange == "engine" else
                               f" (torch.distributed {'RCCL' if args.dist_backend == 'nccl' else 'gloo, host-staged'})")
                            if world > 1 else "single GPU") + f"; {args.inflight} batches in flight",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "ivf_screen_collect" if deferred else ("ivf_scan_screen" if screened else "ivf_scan_wide"),
            "bytes_model": ((("deferred screen, collect kernel: dp B int8 shadow + 4 B scale" if shadow_i8 else
                              "deferred screen, collect kernel: 2 dp B bf16 shadow") +
                             " + 16 B norms per vector of the distinct probed lists + 16 B per collected (query, vector) "
                             "candidate") if deferred else
                            "screened: 2 dp B bf16 shadow + 16 B norms per vector of the distinct probed lists "
                            "+ 4 dp B per exactly re-checked (query, vector) pair" if screened else
                            "exact: 4 D B per vector of the distinct probed lists"),
            "kernel_ms_per_launch": round(kernel_ms, 4),
            "fp32_list_bytes_per_batch": int(fp32_bytes),
            "fp32_equivalent_GBps": round(fp32_bytes / (scan_ms * 1e-3) / 1e9, 1) if scan_ms > 0 else None,
            # SURVEY 8(d)'s model (4 D B per vector of the distinct probed lists) over the whole scan
            # phase: above 1 where the kernel reads the half-size shadow instead of the fp32 lists
            "frac_fp32_model": round(fp32_bytes / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if scan_ms > 0 else None,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_note,
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "scan_ms_per_launch": round(scan_ms, 4),
            "coarse_ms_per_batch": round(prof["coarse_ms"] / launches, 4),
            "search_ms_per_batch": round(prof["total_ms"] / launches, 4),
            "distinct_lists_per_batch": round(prof["distinct_lists"] / max(prof["batches"], 1), 1),
            "distances_per_batch": int(prof["pair_vectors"] / max(prof["batches"], 1)),
            **({"exact_reranks_per_batch": int(prof["exact_reranks"] / max(prof["batches"], 1)),
                "bounded_blocks_per_batch": int(prof["bounded_blocks"] / max(prof["batches"], 1))}
               if prof.get("bounded_blocks") else {}),
            **({"collected_per_batch": int(prof.get("screen_collected", 0) / batches),
                "recheck_ms_per_batch": round(prof.get("recheck_ms", 0.0) / launches, 4),
                "recheck_bytes_per_batch": int(prof["exact_reranks"] / batches * 4 * dp)} if deferred else {}),
        },
        "footprint": footprint(idx, args, world),
        "build": build_info,
        **({"list_cache": idx.cache_stats()} if any(o.startswith("list_cache_bytes=") for o in args.opt) else {}),
        "engine_options": dict(o.split("=", 1) for o in args.opt),
        **({"rehearsal": f"{world} ranks on {torch.cuda.device_count()} GPU(s), host-staged exchange: "
                         "protocol check, not a scaling number"} if args.rehearsal else {}),
        **({"emulated_shard": f"rank {er} of {args.emulate_shard} (partial results; diagnostic, not a bench line)"}
           if args.emulate_shard > 1 else {}),
    }
    if res["per_rank"]:
        result["per_rank"] = res["per_rank"]
        result["rank_balance"] = balance(res["per_rank"])
    if parity_multi is not None:
        result["parity_vs_single_gpu"] = {"batches": min(args.check_batches, args.steps), "bit_identical": parity_multi}
    if args.host_api and world == 1:
        result["host_api"] = host_api_leg(idx, args, queries, out_d, out_i)
    if world == 1 and rank == 0 and not args.no_cpu and args.emulate_shard <= 1:
        qh = queries[: args.cpu_queries].cpu().numpy()
        result["cpu_baseline"] = cpu_baseline(vdb, idx, args, qh, args.cpu_budget)
        result["timed_batch_parity"] = timed_batch_parity(idx, args, queries, out_d, out_i)
    if world == 1 and args.emulate_shard > 1 and args.shard_check > 0:
        qh = queries[: args.shard_check].cpu().numpy()
        result["shard_parity"] = shard_parity(vdb, idx, args, qh, er, args.emulate_shard)
    if args.tier_cache_gib > 0 and world == 1:  # (last: it releases the HBM-resident index)
        tq = torch.empty((args.tier_call * args.tier_calls, args.dim), dtype=torch.float32, device=device)
        fill_rows(vdb, args, tq, 1 << 40, tq.shape[0], 12346, torch.cuda.current_stream().cuda_stream)
        result["tier"] = tier_leg(vdb, idx, args, device, tq)
        idx = None
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
