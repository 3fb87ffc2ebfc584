#!/bin/bash
# select-phase grid 4096 (in-tree) vs 1024, and the 32-query items' threshold refresh on cfg4
set -o pipefail
bash tools/r4_gpu.sh r5ai "s:cfg4:|screen_thr_every=1|screen_thr_every=2|inflight=3|inflight=3,screen_thr_every=1@s:cfg3:inflight=2@s:s8:inflight=3" || exit $?
VDB_IVF_LIB=$PWD/_variants/sel1024/libvdb_ivf.so bash tools/r4_gpu.sh r5ai_sel1024 "s:cfg4:|inflight=3@s:cfg3:inflight=2@s:s8:inflight=3"
