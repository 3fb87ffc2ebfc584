set -o pipefail
O=gpurun_out/scr10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in cfg3 mix cfg4; do
timeout -k 10 700 python -u tools/knob_sweep.py $w "" "segs_per_item=4" "segs_per_item=16" > $O/$w.log 2>&1 || exit $?
grep '^{' $O/$w.log
done
