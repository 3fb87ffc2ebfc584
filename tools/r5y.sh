#!/bin/bash
# collect epilogue without returning global accesses: parity tests, then same-box A/B against
# the previous build (_variants/head) on the headline and the 1/8 shard
set -o pipefail
bash tools/r4_gpu.sh r5y "t:tests/test_gpu_screen.py;tests/test_gpu_screen_tier.py;tests/test_gpu_parity.py@s:cfg3:|inflight=2@s:s8:|inflight=3@s:mix:" || exit $?
VDB_IVF_LIB=$PWD/_variants/head/libvdb_ivf.so bash tools/r4_gpu.sh r5y_head "s:cfg3:|inflight=2@s:s8:|inflight=3@s:mix:"
