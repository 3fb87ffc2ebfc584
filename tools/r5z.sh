#!/bin/bash
# after the collect-epilogue change: the 1/8-shard timeline at 3 in flight, and the knobs whose
# balance it may have moved (grid size, segments per item, shadow format) on cfg3 / s8 / cfg4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --emulate-shard 8 --inflight 3 --steps 100 --warmup 10 --no-cpu --latency-batches 0 > $O/b_s8.log 2>&1 || exit $?
f=$(find $O/tr -name '*kernel_trace.csv' | head -1); python3 tools/timeline.py $f 100 > $O/tr.timeline.json; head -40 $O/tr.timeline.json
grep -h '^{' $O/b_s8.log | cut -c1-300
bash tools/r4_gpu.sh r5z "s:s8:inflight=3|inflight=3,scan_blocks=256|inflight=3,scan_blocks=384|inflight=3,scan_blocks=512|inflight=3,segs_per_item=8|inflight=3,screen_i8=0@s:cfg3:inflight=2|inflight=2,scan_blocks=384|inflight=2,scan_blocks=512|inflight=2,segs_per_item=4|inflight=2,segs_per_item=16|inflight=2,screen_i8=0@s:cfg4:|screen_i8=1|scan_blocks=256,screen_i8=1"
