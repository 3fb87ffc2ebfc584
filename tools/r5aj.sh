#!/bin/bash
# workspace slots 4 / 5 with as many batches in flight (1/8 shard, cfg3), and the smoke entry point
set -o pipefail
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5aj_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5aj_smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_gpu.sh r5aj_s3 "s:s8:inflight=3|inflight=3@s:cfg3:inflight=2|inflight=3" || exit $?
VDB_IVF_LIB=$PWD/_variants/slots4/libvdb_ivf.so bash tools/r4_gpu.sh r5aj_s4 "s:s8:inflight=3|inflight=4|inflight=4@s:cfg3:inflight=3|inflight=4" || exit $?
VDB_IVF_LIB=$PWD/_variants/slots5/libvdb_ivf.so bash tools/r4_gpu.sh r5aj_s5 "s:s8:inflight=4|inflight=5|inflight=5"
