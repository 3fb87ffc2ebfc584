#!/bin/bash
# slot streams: the GPU suite (without the large-config files), then the 1/8 shard's in-flight
# step repeated with slot_streams 1 (default) and 0, cfg3 at 2 in flight, the bench line
set -o pipefail
T=$(ls tests/test_gpu_*.py | grep -v large_configs | tr '\n' ';')
bash tools/r4_gpu.sh r5ac "t:$T@s:s8:inflight=3|inflight=3|inflight=3|inflight=3|inflight=3,slot_streams=0|inflight=3,slot_streams=0|inflight=3,slot_streams=0|inflight=3,slot_streams=0@s:cfg3:inflight=2|inflight=2,slot_streams=0|inflight=2|inflight=2,slot_streams=0@b:--emulate-shard;8;--inflight;3;--steps;200;--warmup;20;--no-cpu;--latency-batches;0"
