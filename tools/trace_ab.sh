#!/bin/bash
# Kernel-trace averages of the headline bench (one batch in flight) per library build.
#   usage: bash tools/trace_ab.sh <tag> <variant or -> ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for L in "$@"; do
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; N=intree; else export VDB_IVF_LIB=$PWD/_variants/$L/libvdb_ivf.so; N=$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$N -o k -f csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --inflight 1 > $O/$N.log 2>&1 || { tail -5 $O/$N.log; exit 1; }
  unset VDB_IVF_LIB
  python3 - "$O/$N/k_kernel_stats.csv" "$N" <<'PY'
import csv, sys
for r in csv.reader(open(sys.argv[1])):
    if r[0] != "Name" and any(x in r[0] for x in ["plan", "merge", "rerank", "coarse_mfma<", "carry", "pad_q", "scan_wide"]):
        print(sys.argv[2], r[0].split("(")[0][:40], r[1], round(float(r[3]) / 1000, 1), "us")
PY
done
