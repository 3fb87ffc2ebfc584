set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5t; mkdir -p $O
i=0
run() {
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py --steps 300 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 "$@" > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$*]', d['value'], d['ms_per_step'], 'collect', r['kernel_ms_per_launch'])"
}
for sb in 320 352 384; do run --opt scan_blocks=$sb; done
for sb in 320 352; do run --data mixture --opt scan_blocks=$sb; done
for sb in 288 352; do run --emulate-shard 8 --inflight 3 --opt scan_blocks=$sb; done
