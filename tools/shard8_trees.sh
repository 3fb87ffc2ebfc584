# 1/8-shard emulation (3 in flight) of whole trees built under _variants/<tree>/ (a git
# worktree's bench.py + package + built lib) and of the working tree ("-"), one GPU call.
#   usage: bash tools/shard8_trees.sh <tree or -> ...
set -o pipefail
O=$PWD/gpurun_out/s15; mkdir -p $O
for t in "$@"; do
  if [ "$t" = "-" ]; then d=.; n=head; else d=_variants/$t; n=$t; fi
  (cd $d && timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_$n.log 2>&1) || { tail -5 $O/shard8_$n.log; exit 1; }
  grep '^{' $O/shard8_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n shard8', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'])"
done
