#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE passes over bench.py into HBM bytes per scan
launch, one entry per workload, merged into one JSON file that bench.py reads
(--traffic-json; the bench line's roofline.traffic).

FETCH_SIZE counts the L2's memory-side read requests; on gfx950 it reports exactly half
of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, "HBM"), so the
value is doubled. rocprofv3 reports FETCH_SIZE in KiB. The scan phase of one batch is one
ivf_scan_wide dispatch (plus ivf_scan_narrow when the fused scan is off): the bytes of
all scan dispatches are summed and divided by the number of batches.

Every entry is stamped with the build id of the library it was measured on (vdb_build_id,
a hash of the scan kernel sources); bench.py uses an entry only on a library of that id.

usage: tools/pmc_traffic.py <out.json> (<pmc-output-dir> <batches> <workload-key>)...
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def build_id():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "cuda-acceleratedvectordatabaseengine_amd")
    spec = importlib.util.spec_from_file_location("vdb_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vdb_amd"] = mod  # (dataclasses resolve their module by name)
    spec.loader.exec_module(mod)
    return mod.build_id()


def summarise(d, batches, key):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    per_kernel = defaultdict(float)
    dispatches = defaultdict(set)
    per_dispatch = defaultdict(float)  # (collect kernel, dispatch) -> KiB
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != "FETCH_SIZE":
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            per_kernel[name] += float(row["Counter_Value"])
            dispatches[name].add(row.get("Dispatch_Id", ""))
            if "ivf_screen_collect" in name:
                per_dispatch[(name, row.get("Dispatch_Id", ""))] += float(row["Counter_Value"])
    scan = {k: v for k, v in per_kernel.items() if "ivf_scan" in k or "ivf_screen_collect" in k}
    kib = sum(scan.values())
    # the deferred screen: one collect dispatch per batch, whatever else the command ran; the
    # median dispatch (a screen build's calibration batch of the index's own vectors, and any
    # other odd one, stays out of it)
    ncol = sum(len(v) for k, v in dispatches.items() if "ivf_screen_collect" in k)
    if ncol:
        batches = ncol
        vals = sorted(per_dispatch.values())
        kib_launch = vals[len(vals) // 2]
    else:
        kib_launch = kib / batches
    return {
        "workload": key,
        "build_id": build_id(),
        "hbm_bytes_per_scan_launch": int(kib_launch * 1024.0 * 2.0),
        "source": "rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950 correction) of the ivf_screen_collect dispatches "
                  f"(median of {batches}), else summed over the ivf_scan_* dispatches of {batches} batches",
        "per_kernel_bytes_per_batch": {k: int(v * 2048 / batches) for k, v in scan.items()},
        "dispatches": {k: len(v) for k, v in dispatches.items() if "ivf_scan" in k or "ivf_screen_collect" in k},
    }


def main():
    out, rest = sys.argv[1], sys.argv[2:]
    if len(rest) % 3 or not rest:
        sys.exit(__doc__)
    merged = {"workloads": {}}
    if os.path.exists(out):
        with open(out) as fh:
            old = json.load(fh)
        merged["workloads"].update(old.get("workloads", {}))
        if "workload" in old:  # the round-1 single-workload form
            merged["workloads"][old["workload"]] = old
    for i in range(0, len(rest), 3):
        res = summarise(rest[i], int(rest[i + 1]), rest[i + 2])
        merged["workloads"][res["workload"]] = res
        print(json.dumps(res))
    with open(out, "w") as fh:
        json.dump(merged, fh, indent=1)


if __name__ == "__main__":
    main()
