# One bench line per engine option set (run via gpurun).
#   usage: bash tools/sweep_lines.sh <tag> "<bench args>" "<opt set>" ... ("-" = defaults)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for set in "$@"; do
  i=$((i+1)); OPTS=""
  [ "$set" != "-" ] && for kv in $set; do OPTS="$OPTS --opt $kv"; done
  timeout -k 10 400 python3 -u bench.py --no-cpu $ARGS $OPTS > $O/run$i.log 2>&1 || { tail -20 $O/run$i.log; exit 1; }
  grep '^{' $O/run$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$set]', d['value'], d['ms_per_step'], 'scan', d['roofline']['scan_ms_per_launch'], 'frac', d['roofline']['frac'])"
done
