# 1/8-shard step at several in-flight depths and knobs: bench lines (the ground truth) and the
# knob sweep's in-flight timing on one build (cross-check)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f; mkdir -p $O
B="--emulate-shard 8 --steps 200 --warmup 10 --no-cpu --latency-batches 0 --prof-steps 5"
i=0
for v in "--inflight 3" "--inflight 3 --opt screen_i8=1" "--inflight 3 --opt scan_blocks=256" "--inflight 2" "--inflight 4"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u bench.py $B $v > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v]', d['value'], d['ms_per_step'], 'collect', d['roofline']['kernel_ms_per_launch'])"
done
timeout -k 10 600 python3 -u tools/knob_sweep.py s8 "inflight=3" "inflight=3,screen_i8=1" "inflight=3,scan_blocks=256" "inflight=2" "inflight=4" > $O/sweep.log 2>&1; grep step_ms $O/sweep.log
