# hybrid exact kernel: screen tests, then bench lines bf16 vs int8 (headline, 1/8 shard, mixture)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_screen_tier.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in "" "--opt screen_i8=1" "--emulate-shard 8 --inflight 3" "--emulate-shard 8 --inflight 3 --opt screen_i8=1" "--data mixture" "--data mixture --opt screen_i8=1 --opt screen_floor_ppm=0"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py --steps 200 --warmup 10 --no-cpu --latency-batches 0 --prof-steps 10 $v > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$v]', d['value'], d['ms_per_step'], 'collect', r['kernel_ms_per_launch'], 'scan', r['scan_ms_per_launch'], 'recheck', r.get('recheck_ms_per_batch'), 'fp', d['footprint']['over_fp32_lists'])"
done
