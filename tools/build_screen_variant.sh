#!/bin/bash
# A/B library build of the screened scan: screen.hip compiled with extra -D flags, linked
# with the in-tree kernels / engine objects into _variants/<name>/libvdb_ivf.so (select it
# with VDB_IVF_LIB).   usage: bash tools/build_screen_variant.sh <name> [-DMACRO=value ...]
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cuda-acceleratedvectordatabaseengine_amd
[ -n "$NOMAKE" ] || make -s -C "$P" >/dev/null
O=$R/_variants/$N
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -I$R/include -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $F "$@" -c "${SRC:-$P/csrc/screen.hip}" -I"$P/csrc" -o "$O/screen.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libvdb_ivf.so" "$P/build/kernels.o" "$O/screen.o" "$P/build/screen_post.o" \
    "$P/build/engine.o" "$P/build/group.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$O/screen.o"
echo "$O/libvdb_ivf.so"
