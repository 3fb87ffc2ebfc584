#!/bin/bash
# cfg4 rank-0-of-8 shard bench line with a full-size parity sample against the oracle.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s6; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --cfg cfg4 --emulate-shard 8 --inflight 3 --shard-check 2 --traffic-json gpurun_out/s5/traffic_cfg4.json > $O/cfg4.log 2>&1 || { tail -20 $O/cfg4.log; exit 1; }
grep '^{' $O/cfg4.log > $O/cfg4.json; cut -c1-400 $O/cfg4.json; grep -o '"shard_parity.*' $O/cfg4.json
