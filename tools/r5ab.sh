#!/bin/bash
# the 1/8 shard's 3-in-flight step, one option set repeated (each set takes the next two streams
# of torch's pool): default hardware queues (4) and 8
set -o pipefail
S="s:s8:inflight=3|inflight=3|inflight=3|inflight=3|inflight=3|inflight=3"
bash tools/r4_gpu.sh r5ab "$S" || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/r4_gpu.sh r5ab_q8 "$S"
