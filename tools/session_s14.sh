set -o pipefail
O=$PWD/gpurun_out/s14; mkdir -p $O
(cd _variants/r1tree && timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_r1.log 2>&1) || { tail -5 $O/shard8_r1.log; exit 1; }
grep '^{' $O/shard8_r1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r1 shard8', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'])"
timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_head.log 2>&1 || exit 1
grep '^{' $O/shard8_head.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('head shard8', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'])"
