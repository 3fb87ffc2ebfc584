#!/bin/bash
# PMC FETCH_SIZE of the collect kernel on rank 0's shard of a 2- and 4-GPU headline job, measured on
# one GPU (bench.py --emulate-shard N: the same LPT lists and queries as rank 0 of the N-GPU job),
# keyed N2 / N4 for the driver's multi-GPU bench lines. usage: bash tools/pmc_rank0_traffic.sh
set -o pipefail
O=gpurun_out/fin15; mkdir -p $O; export TMPDIR=/tmp
S="--steps 5 --warmup 1 --no-cpu --prof-steps 2 --latency-batches 0 --inflight 3"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d $O/pmc_s2 -o f -f csv -- python3 bench.py $S --emulate-shard 2 > $O/pmc_s2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d $O/pmc_s4 -o f -f csv -- python3 bench.py $S --emulate-shard 4 > $O/pmc_s4.log 2>&1 && \
python3 tools/pmc_traffic.py $O/traffic.json $O/pmc_s2 8 "10000000x768/4096/32/64/10/N2" $O/pmc_s4 8 "10000000x768/4096/32/64/10/N4" | tail -3
