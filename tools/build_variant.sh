#!/bin/bash
# A/B library build: kernels.hip compiled with extra -D flags, linked with the in-tree
# engine objects into _variants/<name>/libvdb_ivf.so (select it with VDB_IVF_LIB).
#   usage: bash tools/build_variant.sh <name> [-DMACRO=value ...]
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cuda-acceleratedvectordatabaseengine_amd
[ -n "$NOMAKE" ] || make -s -C "$P" >/dev/null
O=$R/_variants/$N
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -I$R/include"
/opt/rocm/bin/hipcc $F "$@" -c "${SRC:-$P/csrc/kernels.hip}" -I"$P/csrc" -o "$O/kernels.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libvdb_ivf.so" "$O/kernels.o" "$P/build/screen.o" "$P/build/screen_post.o" "$P/build/engine.o" \
    "$P/build/group.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$O/kernels.o"
echo "$O/libvdb_ivf.so"
