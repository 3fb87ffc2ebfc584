# Bench lines per library build (VDB_IVF_LIB), run via gpurun.
#   usage: bash tools/ab_libs.sh <tag> "<bench args>" <lib or -> ...   (- = the in-tree build)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1))
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/$L; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu $ARGS > $O/run$i.log 2>&1 || { tail -20 $O/run$i.log; exit 1; }
  grep '^{' $O/run$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$L]', d['value'], d['ms_per_step'], 'scan', d['roofline']['scan_ms_per_launch'], 'frac', d['roofline']['frac'])"
done
unset VDB_IVF_LIB
