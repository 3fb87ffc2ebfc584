# kernel stats of the cfg3 collect + recheck chain, bf16 vs int8 shadow (one batch in flight)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h; mkdir -p $O
for v in "screen_i8=0" "screen_i8=1"; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 -u tools/knob_sweep.py cfg3 "$v" > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep '^{' $O/$v.log | cut -c1-300
  f=$(find $O/$v -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name'].split('(')[0].replace('void ', '').replace('vdbk::', '')
    if 'screen' in n or 'merge' in n or 'coarse_mfma<' in n or 'select_rerank' in n or 'plan' in n:
        print(f"  {n[:50]:50s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
