set -o pipefail
O=gpurun_out/scr17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in cfg3 mix; do
timeout -k 10 700 python -u tools/knob_sweep.py $w "" > $O/$w.log 2>&1 || exit $?
grep '^{' $O/$w.log
done
run() { name=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu --steps 80 --emulate-shard 8 --inflight 3 "$@" > $O/$name.log 2>&1 || exit $?
  grep '^{' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], d['p99_ms'], r['scan_ms_per_launch'], r['search_ms_per_batch'], r.get('exact_reranks_per_batch'))"; }
run emu8
timeout -k 10 700 python -u tools/knob_sweep.py cfg4 "" > $O/cfg4.log 2>&1 || exit $?
grep '^{' $O/cfg4.log
