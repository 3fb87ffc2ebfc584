#!/bin/bash
# The round's measured evidence, in dependency order (run via gpurun from the repo root):
# PMC HBM bytes of the scan first (the bench line's roofline.traffic reads them), then the
# headline bench line, the 1/8-shard emulation, a batch-512 line, and the kernel-trace
# summary of the one-in-flight bench command. Every GPU step has its own time limit.
#   usage: bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
KEY="10000000x768/4096/32/64/10/N1"
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ivf_scan_ -d "$O/pmc_f" -o f -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2
python3 tools/pmc_traffic.py "$O/pmc_f" 8 "$KEY" "$O/traffic.json" | head -4
run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-include-regex ivf_scan_ -d "$O/pmc_s" -o s -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2
run bench 400 python3 -u bench.py --traffic-json "$O/traffic.json"
grep '^{' "$O/bench.log" > "$O/bench.json" && cut -c 1-300 "$O/bench.json"
run shard 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3
grep '^{' "$O/shard.log" > "$O/shard.json"
run batch512 300 python3 -u bench.py --no-cpu --batch 512 --steps 30
grep '^{' "$O/batch512.log" > "$O/batch512.json"
run prof 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o k -f csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --inflight 1
find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;
head -8 "$O/kernel_stats.csv"
echo "profile_round $TAG done"
