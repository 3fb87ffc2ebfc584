# 1/8-shard knobs at 3 in flight (int8 automatic), then every rank with the emulated exchange
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5o; mkdir -p $O
i=0
for v in "" "--opt scan_blocks=256" "--opt scan_blocks=384" "--inflight 4"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py --emulate-shard 8 --inflight 3 --steps 300 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 $v > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$v]', d['value'], d['ms_per_step'], 'collect', r['kernel_ms_per_launch'], 'scan', r['scan_ms_per_launch'])"
done
timeout -k 10 1500 python3 -u bench.py --emulate-rank all --steps 200 --warmup 20 --latency-batches 0 > $O/ranks.log 2>&1 || { tail -20 $O/ranks.log; exit 1; }
grep '^{"metric"' $O/ranks.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for r in d['ranks']: print(r['rank'], r['ms_per_step'], r['scan_ms'], r['exchange_wait_ms'], r['rank_merge_ms'])
print(d['balance']['ms_per_step'], d['predicted_8gpu_qps_from_max_rank_step'])"
