#!/bin/bash
# collect depth (k-steps in flight per wave, 16-query int8 items): in-tree 4 vs 6 / 3 / 2
set -o pipefail
S="s:cfg3:inflight=2@s:s8:inflight=3"
bash tools/r4_gpu.sh r5ah_kd4 "$S" || exit $?
for v in kd6 kd3 kd2; do VDB_IVF_LIB=$PWD/_variants/$v/libvdb_ivf.so bash tools/r4_gpu.sh r5ah_$v "$S" || exit $?; done
