#!/bin/bash
# PMC FETCH_SIZE of the exact re-check kernel (lane per survivor) at the headline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ao; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_screen_exact" -d $O/pmc -o f -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 --latency-batches 0 > $O/b.log 2>&1 || exit $?
f=$(find $O/pmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, statistics, collections
v = collections.defaultdict(float)
name = {}
for r in csv.DictReader(open(sys.argv[1])):
    v[r['Dispatch_Id']] += float(r['Counter_Value'])
    name[r['Dispatch_Id']] = r['Kernel_Name'].split('(')[0]
by = collections.defaultdict(list)
for d, x in v.items():
    by[name[d]].append(x * 1024 * 2)
for n, xs in by.items():
    print(n, 'dispatches', len(xs), 'median bytes', statistics.median(xs))
PY
