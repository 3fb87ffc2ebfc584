#!/usr/bin/env python3
"""MFMA evidence for the matrix-core kernels: joins a rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...) with a --kernel-trace
pass of the same command. Per kernel: dispatches, median and mean duration, MFMA-busy
fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs) — the
derived MfmaUtil of rocprofv3 -L with GRBM_GUI_ACTIVE taken per XCD (the collected value
sums the 8 XCDs' copies: it is 8x the dispatch's shader-clock cycles) — and for the MFMA
kernels the f32 FLOP rate from the launch shape (2 x rows x centroids x padded dim per
dispatch, rows and centroids read off the grid: one wave = 16 x 16 (ivf_coarse_mfma) or
32 x 32 (ivf_coarse_mfma2x2) outputs) against the 157.3 TF/s f32-MFMA peak.

usage: tools/mfma_report.py <pmc-dir> <trace-dir> [out.json] [--dp 768]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
PEAK_F32_MFMA = 157.3e12


def rows(d, pattern):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        yield from csv.DictReader(open(f))


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    pmc_dir, trace_dir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else None
    dp = int(sys.argv[sys.argv.index("--dp") + 1]) if "--dp" in sys.argv else 768
    ctr = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in rows(pmc_dir, "*counter_collection.csv"):
        k = short(r["Kernel_Name"])
        ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    dur = defaultdict(list)
    flops = defaultdict(float)
    for r in rows(trace_dir, "*kernel_trace.csv"):
        k = short(r["Kernel_Name"])
        ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        dur[k].append(ns)
        gx, gy = int(r.get("Grid_Size_X", 0) or 0), int(r.get("Grid_Size_Y", 0) or 0)
        if "ivf_coarse_mfma2x2" in k:
            flops[k] += 2.0 * (gy * 32) * (gx // 64 * 32) * dp
        elif "ivf_coarse_mfma" in k:
            flops[k] += 2.0 * (gy * 16) * (gx // 64 * 16) * dp
    res = {}
    for k in sorted(set(ctr) | set(dur)):
        c = ctr.get(k, {})
        n = max(len(disp.get(k, ())), 1)
        e = {"dispatches_pmc": len(disp.get(k, ())), "dispatches_trace": len(dur.get(k, ()))}
        if dur.get(k):
            sd = sorted(dur[k])
            e["avg_us"] = round(sum(sd) / len(sd) / 1e3, 2)
            e["median_us"] = round(sd[len(sd) // 2] / 1e3, 2)
        if c.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_frac"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS), 4)
        for name in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"):
            if name in c:
                e[name + "_per_dispatch"] = round(c[name] / n)
        if flops.get(k) and dur.get(k):  # (a median dispatch: the first one carries lazy code loading)
            med = sorted(dur[k])[len(dur[k]) // 2]
            tf = flops[k] / len(dur[k]) / (med * 1e-9)
            e["tflops_f32"] = round(tf / 1e12, 2)
            e["frac_of_f32_mfma_peak"] = round(tf / PEAK_F32_MFMA, 4)
        res[k] = e
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as fh:
            json.dump({"source": "rocprofv3 --pmc + --kernel-trace of the same bench command", "kernels": res}, fh,
                      indent=1)


if __name__ == "__main__":
    main()
