#!/bin/bash
# A/B library: the per-batch chain's short kernels (kernels.hip, screen_post.hip) built with
# -DVDB_CHAIN_PRIO=<p> (s_setprio over the collect kernel's waves), linked with the in-tree
# collect (screen.o) and engine into _variants/prio<p>/libvdb_ivf.so (select it with VDB_IVF_LIB).
#   usage: bash tools/build_chain_prio_variant.sh <p>
set -e
PR=${1:-2}
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cuda-acceleratedvectordatabaseengine_amd
O=$R/_variants/prio$PR
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -I$R/include -DVDB_CHAIN_PRIO=$PR"
/opt/rocm/bin/hipcc $F -c "$P/csrc/kernels.hip" -o "$O/kernels.o" &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-atomic-optimizer-strategy=None -c "$P/csrc/screen_post.hip" -o "$O/screen_post.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libvdb_ivf.so" "$O/kernels.o" "$P/build/screen.o" "$O/screen_post.o" \
    "$P/build/engine.o" "$P/build/group.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$O/kernels.o" "$O/screen_post.o"
echo "$O/libvdb_ivf.so"
