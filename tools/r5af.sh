#!/bin/bash
# in-flight streams on dedicated hardware queues: repeated sets no longer alternate?
set -o pipefail
bash tools/r4_gpu.sh r5af "s:s8:inflight=3|inflight=3|inflight=3|inflight=3|inflight=4@s:cfg3:inflight=2|inflight=2|inflight=3@b:--emulate-shard;8;--inflight;3;--steps;200;--warmup;20;--no-cpu;--latency-batches;0@b:--steps;50;--warmup;5;--no-cpu;--latency-batches;0"
