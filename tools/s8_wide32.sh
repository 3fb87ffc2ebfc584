#!/bin/bash
# 32-query wide items: parity, cfg4-shard sweep, cfg3 headline with and without.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s8; mkdir -p $O; export TMPDIR=/tmp
true
true
timeout -k 10 500 python3 -u tools/cfg4_sweep.py "" "wide_group=32" "wide_group=32,segs_per_item=16" "wide_group=32,diag=2" "wide_group=32,diag=1" "wide_group=32,narrow_blocks=32" "wide_group=32,wide_stride=40009" "" > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
grep '^{' $O/sweep.log
for wg in 16 32; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --opt wide_group=$wg > $O/cfg3_$wg.log 2>&1 || { tail -20 $O/cfg3_$wg.log; exit 1; }
  grep '^{' $O/cfg3_$wg.log | cut -c 150-330
done
