#!/usr/bin/env python3
"""Knob sweep (one build, many timings) on a bench workload.

Builds the workload's index once (bench.build_index / build_index_sharded), then times
the scan for each engine option set (HIP events of the engine's profile, one batch in
flight) and the wall time per batch. Options never change results (the result-changing
timing experiments are separate builds: tools/build_variant.sh -DVDB_SCAN_DIAG=n, selected
with VDB_IVF_LIB).
usage: tools/knob_sweep.py cfg3|cfg4|mix "wide_group=32" "seg_vectors=1024,segs_per_item=8" ...
  cfg4 = rank 0 of the 8-way sharded 100M x 768 index (the per-GPU work of 8 GPUs);
  ip = the cfg3 index with the inner-product metric; s8 = rank 0 of the cfg3 index cut 8 ways
  (the per-GPU work of the 8-GPU headline); cancel = the screen's cancellation regime at 2M
  vectors (test_gpu_screen.py's tiny ball far from the origin, 128-D, two lists whose
  centroids are far from the ball: every pair a candidate), nprobe 2
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

DEFAULTS = {"seg_vectors": 0, "segs_per_item": 0, "wide_stride": 1, "fused_scan": 1, "narrow_blocks": 64,
            "wide_group": 16, "fused_merge": 1, "scan_window": 0, "screen": 1, "bounded_stats": 0, "screen_group": 0,
            "screen_defer": 1, "screen_cand_cap": 4 << 20, "screen_floor_ppm": 50000, "screen_thr_every": 0, "screen_i8": 2,
            "collect_stamps": 0, "scan_blocks": 0, "screen_recheck2": 1}


def main():
    wl, sets = sys.argv[1], sys.argv[2:] or [""]
    big = wl == "cfg4"
    args = bench.argparse.Namespace(dim=768, nvec=100_000_000 if big else 10_000_000, nlist=16384 if big else 4096,
                                    nprobe=64 if big else 32, batch=64, k=10, train=100_000, build_chunk=10_000_000,
                                    data="mixture" if wl == "mix" else "iid", mix_components=0, mix_group=0,
                                    mix_spread=0.35, mix_sigma=0.1, metric="ip" if wl == "ip" else "l2")
    vdb = bench.load_vdb()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if wl == "cancel":
        return cancel(vdb, dev, sets)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        if args.data == "mixture":
            args.centers = bench.mixture_centers(vdb, args.nlist, args.nprobe, args.dim, args.mix_spread, dev)
        if big:
            idx, _ = bench.build_index_sharded(vdb, args, dev, 0, 8)
        else:
            idx, _ = bench.build_index(vdb, args, dev, 0, 1)
            if wl == "s8":
                idx.set_shard(0, 8)
        st = torch.cuda.current_stream()
        B, steps, nqb = 64, 12, 128  # (nqb distinct query batches for the in-flight timing)
        q = torch.empty((nqb * B, 768), dtype=torch.float32, device=dev)
        bench.fill_rows(vdb, args, q, 0, nqb * B, 12346, st.cuda_stream)
        od = torch.empty((B, 1024), dtype=torch.float32, device=dev)
        oi = torch.empty((B, 1024), dtype=torch.int64, device=dev)
        ded = {}
        for s in sets:
            opts = [o.split("=") for o in s.split(",") if o]
            kk, infl = 10, 1  # ("k=N", "inflight=N" in a set: the search's k, batches in flight; not engine options)
            for n, v in opts:
                if n == "k":
                    kk = int(v)
                elif n == "inflight":
                    infl = int(v)
                else:
                    idx.set_option(n, int(v))
            opts = [(n, v) for n, v in opts if n not in ("k", "inflight")]
            stamps = any(n == "collect_stamps" for n, _ in opts)
            for j in range(2):
                idx.search_device(q[j * B:].data_ptr(), B, args.nprobe, kk, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            idx.profile_enable(True)
            idx.set_option("bounded_stats", 1)  # statistics only
            idx.profile_reset()
            t0 = time.perf_counter()
            for j in range(steps):
                idx.search_device(q[j * B:].data_ptr(), B, args.nprobe, kk, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / steps * 1e3
            p = idx.profile_read()
            idx.profile_enable(False)
            if stamps:
                rec, hz = idx.collect_stamps()
                print(json.dumps(dict(stamp_summary(rec, hz), workload=wl, opts=s)), flush=True)
            n = max(p["scan_launches"], 1)
            alg = p["scan_bytes"] / max(p["batches"], 1)
            print(json.dumps({"workload": wl, "opts": s, "gpu_bytes": idx.gpu_bytes_allocated(), "scan_ms": round(p["scan_ms"] / n, 3),
                              "search_ms": round(p["total_ms"] / n, 3), "wall_ms": round(wall, 3),
                              "alg_GB": round(alg / 1e9, 2),
                              "pairs_M": round(p["pair_vectors"] / max(p["batches"], 1) / 1e6, 2),
                              "computed_M": round(p["computed_vectors"] / max(p["batches"], 1) / 1e6, 2), "frac": round(alg / (p["scan_ms"] / n * 1e-3) / 8e12, 4),
                              "rechecks_M": round(p["exact_reranks"] / max(p["batches"], 1) / 1e6, 3),
                              "collected_M": round(p.get("screen_collected", 0) / max(p["batches"], 1) / 1e6, 3),
                              "collect_ms": round(p.get("collect_ms", 0) / n, 3),
                              "recheck_ms": round(p.get("recheck_ms", 0) / n, 3)}),
                  flush=True)
            if infl > 1:  # the step at `infl` batches in flight (round-robin streams, as bench.py)
                idx.set_option("bounded_stats", 0)
                if infl not in ded:  # (a hardware queue each, created once per depth)
                    ded[infl] = bench.dedicated_streams(dev, infl)
                streams = ded[infl]
                nb = 100
                for j in range(nb + 6):
                    if j == 6:
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                    s_ = streams[j % infl]
                    idx.search_device(q[(j % nqb) * B:].data_ptr(), B, args.nprobe, kk, od.data_ptr(), oi.data_ptr(),
                                      s_.cuda_stream)
                t_sub = time.perf_counter()  # (host time to submit the nb calls: the GPU starves when it nears the step)
                torch.cuda.synchronize()
                print(json.dumps({"workload": wl, "opts": s, "inflight": infl,
                                  "step_ms": round((time.perf_counter() - t0) / nb * 1e3, 4),
                                  "submit_ms_per_call": round((t_sub - t0) / nb * 1e3, 4)}), flush=True)
            for n_, _ in opts:  # back to defaults
                idx.set_option(n_, DEFAULTS[n_])


def stamp_summary(rec, hz):
    """The collect kernel's timeline (option collect_stamps) per batch: the workgroups' start
    ramp, the span, the wide items' share of the workgroup-time, the tail after the last
    item started, and the slowest items."""
    import numpy as np
    if not len(rec):
        return {"stamps": 0}
    us = 1e6 / hz
    batch = (rec[:, 0] >> np.uint64(40)).astype(np.int64)
    kind = ((rec[:, 3] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.int64)
    nq = (rec[:, 3] & np.uint64(0xFF)).astype(np.int64)
    segs = ((rec[:, 3] >> np.uint64(8)) & np.uint64(0xFF)).astype(np.int64)
    t0 = rec[:, 1].astype(np.float64)
    t1 = rec[:, 2].astype(np.float64)
    out = []
    for b in np.unique(batch)[1:]:  # (the first batch warms up)
        m = batch == b
        st, wi, na = m & (kind == 2), m & (kind == 0), m & (kind == 1)
        if not st.any() or not wi.any():
            continue
        first, last_start = t0[st].min(), t0[st].max()
        end = max(t1[wi].max(), t1[na].max() if na.any() else 0)
        span = end - first
        dur = t1[wi] - t0[wi]
        nwg = int(st.sum())
        top = np.argsort(-dur)[:3]
        out.append({"span_us": span * us, "wg_start_ramp_us": (last_start - first) * us,
                    "last_wide_item_start_us": (t0[wi].max() - first) * us,
                    "tail_after_last_start_us": (end - t0[wi].max()) * us,
                    "wide_items": int(wi.sum()), "narrow_items": int(na.sum()), "workgroups": nwg,
                    "wide_busy_frac": float(dur.sum() / (nwg * span)),
                    "item_us_mean": float(dur.mean() * us), "item_us_max": float(dur.max() * us),
                    "slowest": [[int(nq[wi][i]), int(segs[wi][i]), round(float(dur[i] * us), 1)] for i in top],
                    "narrow_us_sum": float((t1[na] - t0[na]).sum() * us) if na.any() else 0.0})
    keys = [k for k in out[0] if k != "slowest"] if out else []
    return {"stamp_batches": len(out), **{k: round(float(np.mean([o[k] for o in out])), 2) for k in keys},
            "slowest_items_of_first_batch[nq,segs,us]": out[0]["slowest"] if out else None}


def cancel(vdb, dev, sets):
    """The cancellation regime (the bound wider than the whole distance spread) at 2M x 128."""
    dim, n, B, steps = 128, 2_000_000, 64, 1000
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    c = torch.full((dim,), 100.0 / dim ** 0.5, device=dev)
    X = (c + 0.01 * torch.randn((n, dim), generator=g, device=dev)).contiguous()
    Q = (c + 0.01 * torch.randn(((steps + 2) * B, dim), generator=g, device=dev)).contiguous()
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    idx = vdb.IVFFlatIndex(vdb.IVFFlatIndex.Config(dim, 2, max_gpu_memory=0))
    idx.centroids = torch.stack([torch.zeros_like(c), -c]).cpu().numpy()
    idx.add_device(X.data_ptr(), ids.data_ptr(), n)
    st = torch.cuda.current_stream()
    od = torch.empty((B, 10), dtype=torch.float32, device=dev)
    oi = torch.empty((B, 10), dtype=torch.int64, device=dev)
    ref = None
    for s in sets:
        opts = [o.split("=") for o in s.split(",") if o]
        for nm, v in opts:
            idx.set_option(nm, int(v))
        for j in range(2):
            idx.search_device(Q[j * B:].data_ptr(), B, 2, 10, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        p0 = idx.profile_read()
        t0 = time.perf_counter()
        for j in range(steps):
            idx.search_device(Q[(j + 2) * B:].data_ptr(), B, 2, 10, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e3
        p = idx.profile_read()
        same = None
        if ref is None:
            ref = (od.clone(), oi.clone())
        else:
            same = bool(torch.equal(oi, ref[1]) and torch.equal(od.view(torch.int32), ref[0].view(torch.int32)))
        print(json.dumps({"workload": "cancel", "opts": s, "wall_ms": round(wall, 3),
                          "floor_batches": p["screen_floor_batches"] - p0["screen_floor_batches"],
                          "floor_trips": p["screen_floor_trips"] - p0["screen_floor_trips"],
                          "same_results_as_first": same}), flush=True)
        for nm, _ in opts:
            idx.set_option(nm, DEFAULTS[nm])


if __name__ == "__main__":
    main()
