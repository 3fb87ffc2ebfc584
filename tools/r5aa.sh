#!/bin/bash
# the 1/8 shard's in-flight step with host submit time (repeats: its spread), cfg4 with the
# automatic shadow now int8 for 32-query items
set -o pipefail
bash tools/r4_gpu.sh r5aa "s:s8:inflight=2|inflight=3|inflight=3|inflight=3,scan_blocks=256|inflight=3,scan_blocks=256|inflight=3,screen_i8=0@s:cfg4:|inflight=3"
