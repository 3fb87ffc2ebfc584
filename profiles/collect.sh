# Profiling recipe (run on the GPU box from the repo root): HBM traffic (FETCH_SIZE) and SQ
# stall counters for ivf_scan in separate --pmc passes, then the kernel-trace summary.
# usage: bash profiles/collect.sh <outdir-under-gpurun_out> [bench args...]
O=${1:-pmc}; shift; ARGS="${@:---steps 5 --warmup 1 --no-cpu}"
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$O
mkdir -p $D && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ivf_scan_ -d $D/f -o f -f csv -- python3 $R/bench.py $ARGS > $D/f.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex ivf_scan_ -d $D/s -o s -f csv -- python3 $R/bench.py $ARGS > $D/s.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/k -o k -f csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $D/k.log 2>&1
