# A/B of the bounded wide scan (run via gpurun): bench lines per engine option set.
#   usage: bash tools/ab_bounded.sh <tag> "<cfg args>" "<opt set 1>" "<opt set 2>" ...
#   (an opt set is space-separated NAME=VALUE pairs; "-" = defaults)
set -o pipefail
TAG=$1; CFG=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for set in "$@"; do
  i=$((i+1))
  OPTS=""; [ "$set" != "-" ] && for kv in $set; do OPTS="$OPTS --opt $kv"; done
  timeout -k 10 400 python -u bench.py $CFG --no-cpu --steps 40 --warmup 5 $OPTS > $O/run$i.log 2>&1 || { tail -20 $O/run$i.log; exit 1; }
  grep '^{' $O/run$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('[$set]', d['value'], 'scan_ms', r['scan_ms_per_launch'], 'frac', r['frac'], 'dist/batch', r['distances_per_batch'], 'rerank/batch', r.get('exact_reranks_per_batch'), 'blocks/batch', r.get('bounded_blocks_per_batch'))"
done
