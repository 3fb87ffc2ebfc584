#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ae; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/queue_probe.py > $O/probe.log 2>&1 || exit $?
f=$(find $O/tr -name '*kernel_trace.csv' | head -1); python3 tools/queue_probe_read.py $f $O/probe.log
