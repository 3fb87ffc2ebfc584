#!/bin/bash
# high-priority communicator stream: multi-GPU tests; the 1/8 shard's knobs under stable streams;
# the 1/8-shard line with the emulated 8-record exchange
set -o pipefail
bash tools/r4_gpu.sh r5ag "t:tests/test_gpu_multi.py;tests/test_gpu_tier_shard.py@s:s8:inflight=3|inflight=3,segs_per_item=4|inflight=3,segs_per_item=16|inflight=3,scan_blocks=256|inflight=3,scan_blocks=384|inflight=3,scan_blocks=512@b:--emulate-shard;8;--inflight;3;--steps;200;--warmup;20;--no-cpu;--latency-batches;0;--emulate-exchange"
