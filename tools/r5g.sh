# 1/8-shard step A/B at 3 in flight: chain_priority, int8, scan_blocks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g; mkdir -p $O
B="--emulate-shard 8 --steps 200 --warmup 10 --no-cpu --latency-batches 0 --prof-steps 5 --inflight 3"
i=0
for v in "" "--opt chain_priority=1" "--opt chain_priority=1 --opt scan_blocks=256" "--opt chain_priority=1 --opt screen_i8=1" "--inflight 4 --opt chain_priority=1" ""; do
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py $B $v > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v]', d['value'], d['ms_per_step'], 'collect', d['roofline']['kernel_ms_per_launch'], 'p99_1', d['p99_ms_one_in_flight'])"
done
