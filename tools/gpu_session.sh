#!/bin/bash
# One GPU-box session (run via gpurun from the repo root): parity tests, the default
# bench line, the kernel-trace summary of the bench command, PMC passes.
#   usage: bash tools/gpu_session.sh <tag> [steps, comma-separated:
#          tests,smoke,bench,multi,grpc,prof,pmc]  [extra bench args...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-run}
STEPS=${2:-tests,bench,prof}
shift 2 2>/dev/null
BARGS="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
run() {  # run <name> <seconds> <cmd...>: stop the session on any failure
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    if [ $rc -ne 0 ]; then
        tail -40 "$O/$name.log"
        exit $rc
    fi
}
nproc > "$O/nproc.txt"
lscpu > "$O/lscpu.txt" 2>/dev/null
if has tests; then
    run pytest 1100 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --durations=25 --timeout 600 --timeout-method thread ${PYTEST_K}
    tail -3 "$O/pytest.log"
fi
if has smoke; then
    run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
    tail -2 "$O/smoke.log"
fi
if has bench; then
    run bench 600 python -u bench.py $BARGS
    grep '^{' "$O/bench.log" > "$O/bench.json"
    cat "$O/bench.json"
fi
if has multi; then
    # one-GPU rehearsal of the N-rank path: 2 ranks on cuda:0, gloo exchange staged through host
    # bench.py launches its own ranks (one process per GPU); with one GPU on the box the
    # two ranks share it and exchange through host memory (a protocol rehearsal)
    run multi 600 python -u bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --prof-steps 4
    grep '^{' "$O/multi.log" > "$O/multi.json"
    cat "$O/multi.json"
fi
if has grpc; then
    run grpc 600 python -u tools/grpc_load.py
    grep '^{' "$O/grpc.log" > "$O/grpc.json"
    cat "$O/grpc.json"
fi
if has prof; then
    run prof 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o k -f csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --inflight 1 $BARGS
    find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;
    head -14 "$O/kernel_stats.csv"
fi
if has pmc; then
    # HBM bytes of the scan kernels (FETCH_SIZE; x2 on gfx950, MI355X_MICROARCH.md §HBM)
    run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ivf_scan_ -d "$O/pmc_f" -o f -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 $BARGS
    python3 tools/pmc_traffic.py "$O/pmc_f" 8 "10000000x768/4096/32/64/10/N1" "$O/traffic.json" | head -8
    run pmc_sq 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-include-regex ivf_scan_ -d "$O/pmc_s" -o s -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 $BARGS
fi
echo "session $TAG done"
