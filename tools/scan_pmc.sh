#!/bin/bash
# SQ counters of the scan kernel (issue/stall breakdown) on one bench workload.
#   usage: bash tools/scan_pmc.sh <tag> <name> [bench args...]
set -o pipefail
TAG=$1; NAME=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY"
i=0
for P in "$A" "$B"; do
    i=$((i+1))
    echo "[$(date +%T)] $NAME pass $i"
    timeout -k 10 500 rocprofv3 --pmc $P --kernel-include-regex ${KRE:-ivf_scan_} -d "$O/${NAME}_p$i" -o p -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 "$@" > "$O/${NAME}_p$i.log" 2>&1 || { tail -20 "$O/${NAME}_p$i.log"; exit 1; }
done
python3 - "$O" "$NAME" <<'PY'
import csv, glob, os, sys, collections
o, name = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
for f in glob.glob(os.path.join(o, f"{name}_p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
w = tot["SQ_WAVE_CYCLES"] or 1
print(name, {k: int(v) for k, v in sorted(tot.items())})
print(name, "fractions of wave-cycles:", {k: round(tot[k] / w, 3) for k in
      ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY",
       "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_ANY")})
print(name, "VALU insts per LDS inst:", round(tot["SQ_INSTS_VALU"] / max(tot["SQ_INSTS_LDS"], 1), 2),
      "per VMEM:", round(tot["SQ_INSTS_VALU"] / max(tot["SQ_INSTS_VMEM_RD"], 1), 2))
PY
