set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tr_bf16 -o run -- python3 bench.py --emulate-shard 8 --inflight 3 --steps 100 --warmup 10 --no-cpu --latency-batches 0 > $O/b_bf16.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tr_i8 -o run -- python3 bench.py --emulate-shard 8 --inflight 3 --steps 100 --warmup 10 --no-cpu --latency-batches 0 --opt screen_i8=1 > $O/b_i8.log 2>&1 && \
for d in tr_bf16 tr_i8; do f=$(find $O/$d -name '*kernel_trace.csv' | head -1); python3 tools/timeline.py $f 100 > $O/$d.timeline.json; head -12 $O/$d.timeline.json; done
grep -h '^{' $O/b_*.log | cut -c1-400
