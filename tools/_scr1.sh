set -o pipefail
O=gpurun_out/scr12; mkdir -p $O
export TMPDIR=/tmp
for w in cfg4 mix; do
timeout -k 10 700 python -u tools/knob_sweep.py $w "" "screen_group=16" "screen_group=16,segs_per_item=8" > $O/$w.log 2>&1 || exit $?
grep '^{' $O/$w.log
done
