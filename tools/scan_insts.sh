#!/bin/bash
# Instruction mix of the scan kernel per engine option set (rocprofv3 --pmc over
# tools/knob_sweep.py, 14 scan dispatches per set: 2 warm-up + 12 timed).
#   usage: bash tools/scan_insts.sh <tag> cfg3|cfg4|mix "<opt set>" ...
set -o pipefail
TAG=$1; WL=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
echo "[$(date +%T)] $WL pmc"
timeout -k 10 600 rocprofv3 --pmc $P --kernel-include-regex "ivf_scan_" -d "$O/${WL}_insts" -o p -f csv -- python3 -u tools/knob_sweep.py "$WL" "$@" > "$O/${WL}_insts.log" 2>&1 || { tail -20 "$O/${WL}_insts.log"; exit 1; }
python3 - "$O/${WL}_insts" "$O/${WL}_insts.log" "$@" <<'PY' | tee "$O/${WL}_insts_summary.jsonl"
import csv, glob, os, sys, json, collections
d, log, sets = sys.argv[1], sys.argv[2], sys.argv[3:]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(per)
lines = [json.loads(l) for l in open(log) if l.startswith("{")]
for i, s in enumerate(sets):
    chunk = ids[i * 14 + 2:(i + 1) * 14]
    tot = collections.defaultdict(float)
    for x in chunk:
        for k, v in per[x].items():
            tot[k] += v / len(chunk)
    info = lines[i] if i < len(lines) else {}
    out = {"opts": s or "-", "scan_ms": info.get("scan_ms"), "pairs_M": info.get("pairs_M"),
           "computed_M": info.get("computed_M"), "dispatches": len(chunk)}
    out.update({k: int(v) for k, v in sorted(tot.items())})
    if info.get("pairs_M"):
        hot = info["pairs_M"] * 1e6 * 768 * 1.5 / 64  # packed wave-instructions of the exact sums
        out["valu_over_hot"] = round(tot["SQ_INSTS_VALU"] / hot, 3)
        out["clock_GHz"] = round(tot["GRBM_GUI_ACTIVE"] / 8 / (info["scan_ms"] * 1e-3) / 1e9, 3)
    print(json.dumps(out))
PY
