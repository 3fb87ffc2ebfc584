#!/bin/bash
# knob_sweep lines (two timed repeats each) per library build and workload, in one GPU call.
#   usage: bash tools/ab_sweep.sh <tag> <name>:<variant or ->:<cfg3|cfg4|mix>[:<opt set>] ...
#   (variant = _variants/<variant>/libvdb_ivf.so from tools/build_variant.sh; - = in-tree)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for spec in "$@"; do
  IFS=: read -r name lib wl opts <<< "$spec"
  if [ "$lib" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/_variants/$lib/libvdb_ivf.so; fi
  timeout -k 10 400 python3 -u tools/knob_sweep.py $wl "$opts" "$opts" > $O/$name.jsonl 2>$O/$name.err || { tail -5 $O/$name.err; exit 1; }
  unset VDB_IVF_LIB
  grep -h '^{' $O/$name.jsonl | sed "s/^/[$name] /"
done
