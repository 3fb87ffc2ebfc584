#!/usr/bin/env python3
"""Knob sweep on the cfg4 rank-0-of-8 shard (one build, many timings).

Builds the 100M x 768 / nlist 16384 index's rank-0 shard once (bench.build_index_sharded),
then times the scan for each engine option set (HIP events of the engine's profile,
one batch in flight). Options never change results except diag (timing experiments only).
usage: tools/cfg4_sweep.py "seg_vectors=512" "seg_vectors=1024,segs_per_item=8" ...
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    sets = sys.argv[1:] or [""]
    args = bench.argparse.Namespace(dim=768, nvec=100_000_000, nlist=16384, nprobe=64, batch=64, k=10,
                                    train=100_000, build_chunk=10_000_000)
    vdb = bench.load_vdb()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        idx, _ = bench.build_index_sharded(vdb, args, dev, 0, 8)
        st = torch.cuda.current_stream()
        B, steps = 64, 12
        q = torch.empty((steps * B, 768), dtype=torch.float32, device=dev)
        vdb.gen_normal_device(q.data_ptr(), q.numel(), seed=12346, stream=st.cuda_stream)
        od = torch.empty((B, 10), dtype=torch.float32, device=dev)
        oi = torch.empty((B, 10), dtype=torch.int64, device=dev)
        for s in sets:
            opts = [o.split("=") for o in s.split(",") if o]
            for n, v in opts:
                idx.set_option(n, int(v))
            for j in range(2):
                idx.search_device(q[j * B:].data_ptr(), B, 64, 10, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            idx.profile_enable(True)
            idx.profile_reset()
            t0 = time.perf_counter()
            for j in range(steps):
                idx.search_device(q[j * B:].data_ptr(), B, 64, 10, od.data_ptr(), oi.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / steps * 1e3
            p = idx.profile_read()
            idx.profile_enable(False)
            n = max(p["scan_launches"], 1)
            print(json.dumps({"opts": s, "scan_ms": round(p["scan_ms"] / n, 3), "search_ms": round(p["total_ms"] / n, 3),
                              "wall_ms": round(wall, 3)}), flush=True)
            for n_, _ in opts:  # back to defaults
                idx.set_option(n_, {"seg_vectors": 0, "segs_per_item": 0, "wide_stride": 1, "diag": 0,
                                    "fused_scan": 1, "narrow_blocks": 64, "wide_group": 16}[n_])


if __name__ == "__main__":
    main()
