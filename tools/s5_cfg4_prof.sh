#!/bin/bash
# cfg4 rank-0-of-8 shard: PMC HBM bytes of the scan, then the kernel-trace summary.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s5; mkdir -p $O; export TMPDIR=/tmp
KEY="100000000x768/16384/64/64/10/N1/shard0of8"
A="--cfg cfg4 --emulate-shard 8 --no-cpu"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ivf_scan_ -d $O/pmc_f -o f -f csv -- python3 bench.py $A --steps 5 --warmup 1 --prof-steps 2 > $O/pmc_f.log 2>&1 || { tail -20 $O/pmc_f.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_f 8 "$KEY" $O/traffic_cfg4.json | head -6
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o k -f csv -- python3 bench.py $A --steps 20 --warmup 2 --inflight 1 --traffic-json $O/traffic_cfg4.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
head -8 $O/kernel_stats.csv | cut -c1-200
grep '^{' $O/prof.log | cut -c1-1600
