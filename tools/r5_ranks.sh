#!/bin/bash
# every rank of the 8-GPU headline, a process each, with the emulated 8-record exchange
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 1100 python3 -u bench.py --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu > $O/ranks.log 2>&1
rc=$?; grep '^{' $O/ranks.log | tail -1 > $O/ranks.json; cut -c1-600 $O/ranks.json; tail -5 $O/ranks.log | cut -c1-300; exit $rc
