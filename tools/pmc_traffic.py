#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc FETCH_SIZE pass over bench.py into HBM bytes per batch.

FETCH_SIZE counts the L2's memory-side read requests; on gfx950 it reports exactly half
of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, "HBM"), so the
value is doubled. rocprofv3 reports FETCH_SIZE in KiB.

usage: tools/pmc_traffic.py <pmc-output-dir> <batches> <workload-key> [out.json]
The scan phase of one batch is one ivf_scan_wide dispatch (plus ivf_scan_narrow when the
fused scan is off); the
bytes of all scan dispatches are summed and divided by the number of batches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, batches, key = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else None
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    per_kernel = defaultdict(float)
    dispatches = defaultdict(set)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != "FETCH_SIZE":
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            per_kernel[name] += float(row["Counter_Value"])
            dispatches[name].add(row.get("Dispatch_Id", ""))
    scan = {k: v for k, v in per_kernel.items() if "ivf_scan" in k}
    kib = sum(scan.values())
    bytes_per_batch = kib * 1024.0 * 2.0 / batches
    res = {
        "workload": key,
        "hbm_bytes_per_scan_launch": int(bytes_per_batch),
        "source": "rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950 correction) summed over ivf_scan_wide + "
                  f"ivf_scan_narrow dispatches of {batches} batches",
        "per_kernel_bytes_per_batch": {k: int(v * 2048 / batches) for k, v in scan.items()},
        "dispatches": {k: len(v) for k, v in dispatches.items() if "ivf_scan" in k},
    }
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
