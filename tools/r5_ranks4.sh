#!/bin/bash
# every rank of the 8-GPU configs[3] job (100M x 768, nlist 16384, nprobe 64), a process each,
# with the emulated 8-record exchange
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 1150 python3 -u bench.py --cfg cfg4 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu --steps 50 --warmup 5 > $O/ranks4.log 2>&1
rc=$?; grep '^{' $O/ranks4.log | tail -1 > $O/ranks4.json; cut -c1-400 $O/ranks4.json; tail -3 $O/ranks4.log | cut -c1-300; exit $rc
