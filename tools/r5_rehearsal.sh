#!/bin/bash
# the driver's commands on one GPU: N=1 with its defaults, and the self-launched two-rank rehearsal
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 50 --warmup 5 > $O/driver_n1.log 2>&1 || { tail -20 $O/driver_n1.log; exit 1; }
grep '^{' $O/driver_n1.log | cut -c1-300
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --latency-batches 0 > $O/two_ranks.log 2>&1 || { tail -30 $O/two_ranks.log; exit 1; }
grep '^{' $O/two_ranks.log | cut -c1-400
