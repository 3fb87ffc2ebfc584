# automatic shadow format: the whole GPU suite, then the bench lines (headline, 1/8 shard, mixture)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 1200 python -u -m pytest ${PYT:-tests} -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -12 $O/pytest.log
i=0
for v in "" "--emulate-shard 8 --inflight 3" "--data mixture"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py --steps 200 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 $v > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$v]', d['value'], d['ms_per_step'], 'collect', r['kernel_ms_per_launch'], 'scan', r['scan_ms_per_launch'], 'recheck', r.get('recheck_ms_per_batch'), 'fp', d['footprint']['over_fp32_lists'], r['bytes_model'][:40])"
done
