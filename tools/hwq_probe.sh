# 1/8-shard headline line at several GPU_MAX_HW_QUEUES values (run via gpurun).
set -o pipefail
O=gpurun_out/hwq; mkdir -p $O
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u bench.py --emulate-shard 8 --no-cpu --inflight 3 > $O/q$q.log 2>&1 || { tail -20 $O/q$q.log; exit 1; }
  grep '^{' $O/q$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hwq $q', d['value'], d['ms_per_step'], d['roofline']['scan_ms_per_launch'])"
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u bench.py --no-cpu > $O/cfg3_q8.log 2>&1 || { tail -20 $O/cfg3_q8.log; exit 1; }
grep '^{' $O/cfg3_q8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg3 hwq 8', d['value'], d['ms_per_step'], d['roofline']['scan_ms_per_launch'])"
