set -o pipefail
O=gpurun_out/scr5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_screen.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/knob_sweep.py cfg3 "" > $O/cfg3.log 2>&1 || exit $?
grep '^{' $O/cfg3.log
timeout -k 10 500 python -u tools/knob_sweep.py mix "" > $O/mix.log 2>&1 || exit $?
grep '^{' $O/mix.log
timeout -k 10 700 python -u tools/knob_sweep.py cfg4 "" > $O/cfg4.log 2>&1 || exit $?
grep '^{' $O/cfg4.log
