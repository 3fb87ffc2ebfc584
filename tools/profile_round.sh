#!/bin/bash
# The round's measured evidence (run via gpurun from the repo root), each GPU step under
# its own time limit, stopping at the first failure:
#   traffic  PMC FETCH_SIZE of the scan (x2 gfx950 correction) for the iid headline, the
#            mixture workload and the cfg4 1/8 shard -> gpurun_out/<tag>/traffic.json
#   mfma     SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE of the matrix-core
#            kernels (coarse bounds, 2x2 assignment bounds) and the re-rank / assign kernels
#   bench    the headline line and the mixture line, reading traffic.json
#   trace    rocprofv3 --kernel-trace --stats of the headline bench at 1 and 2 batches in
#            flight, and of the mixture bench
#   shard    the cfg4 rank-0-of-8 shard line (sharded 100M build), with its kernel trace
#   emu8     rank 0 of 8 of the headline index at 3 in flight (the 8-GPU per-GPU work)
#   tier5    the cfg4 rank-0 shard served from a shard file through a smaller HBM cache (cfg5 shape)
#   usage: bash tools/profile_round.sh <tag> [steps, comma-separated]
set -o pipefail
TAG=${1:-round}
STEPS=${2:-traffic,mfma,bench,trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
SHORT="--steps 5 --warmup 1 --no-cpu --prof-steps 2 --latency-batches 0"
# the bench lines read this call's PMC traffic, or the committed file when no traffic step ran
TJ="$O/traffic.json"
[[ ",$STEPS," == *",traffic"* ]] || TJ="$R/profiles/traffic.json"
CFG4="--cfg cfg4 --emulate-shard 8 --no-cpu --inflight 3"
if has traffic; then
    run pmc_iid 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d "$O/pmc_iid" -o f -f csv -- python3 bench.py $SHORT
    run pmc_mix 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d "$O/pmc_mix" -o f -f csv -- python3 bench.py $SHORT --data mixture
    python3 tools/pmc_traffic.py "$O/traffic.json" "$O/pmc_iid" 8 "10000000x768/4096/32/64/10/N1" \
        "$O/pmc_mix" 8 "10000000x768/4096/32/64/10/N1/mixture" | tail -3
fi
if has traffic8; then
    run pmc_emu8 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d "$O/pmc_emu8" -o f -f csv -- python3 bench.py $SHORT --emulate-shard 8 --inflight 3
    python3 tools/pmc_traffic.py "$O/traffic.json" "$O/pmc_emu8" 8 "10000000x768/4096/32/64/10/N1/shard0of8" | tail -3
fi
if has traffic4; then
    run pmc_cfg4 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivf_scan_|ivf_screen_collect" -d "$O/pmc_cfg4" -o f -f csv -- python3 bench.py $CFG4 --steps 5 --warmup 1 --prof-steps 2 --latency-batches 0
    python3 tools/pmc_traffic.py "$O/traffic.json" "$O/pmc_cfg4" 8 "100000000x768/16384/64/64/10/N1/shard0of8" | tail -3
fi
if has mfma; then
    # the bench build's assignment (10M x 4096 bounds on the 2x2 kernel) and the search
    # batches' coarse step; rocprofv3 -L first, for the record of the counters present
    rocprofv3 -L > "$O/counters_available.txt" 2>&1 || true
    run pmc_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "ivf_coarse|ivf_assign|ivf_select_rerank|ivf_screen_collect|ivf_screen_recheck2" -d "$O/pmc_mfma" -o m -f csv -- python3 bench.py $SHORT
    run trace_mfma 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "ivf_coarse|ivf_assign|ivf_select_rerank|ivf_screen_collect|ivf_screen_recheck2" -d "$O/trace_mfma" -o t -f csv -- python3 bench.py $SHORT
    python3 tools/mfma_report.py "$O/pmc_mfma" "$O/trace_mfma" "$O/mfma.json" | tail -30
fi
if has bench; then
    run bench 400 python3 -u bench.py --traffic-json "$TJ" --host-api
    grep '^{' "$O/bench.log" > "$O/bench.json" && cut -c 1-400 "$O/bench.json"
    run bench_mix 400 python3 -u bench.py --traffic-json "$TJ" --data mixture --host-api
    grep '^{' "$O/bench_mix.log" > "$O/bench_mix.json" && cut -c 1-400 "$O/bench_mix.json"
fi
if has trace; then
    for inf in 1 3; do
        run trace_inflight$inf 300 rocprofv3 --kernel-trace --stats -d "$O/trace_inflight$inf" -o k -f csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --inflight $inf --latency-batches 0
        find "$O/trace_inflight$inf" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_inflight$inf.csv" \;
        head -6 "$O/kernel_stats_inflight$inf.csv"
    done
    run trace_mix 300 rocprofv3 --kernel-trace --stats -d "$O/trace_mix" -o k -f csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --inflight 1 --data mixture --latency-batches 0
    find "$O/trace_mix" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_mixture.csv" \;
    head -6 "$O/kernel_stats_mixture.csv"
fi
if has shard; then
    run shard 600 python3 -u bench.py $CFG4 --shard-check 4 --traffic-json "$TJ"
    grep '^{' "$O/shard.log" > "$O/shard.json" && cut -c 1-400 "$O/shard.json"
fi
if has emu8; then
    # rank 0 of 8 cut from the headline index (the per-GPU work of the 8-GPU headline), 3 in flight
    run emu8 600 python3 -u bench.py --emulate-shard 8 --inflight 3 --no-cpu --traffic-json "$TJ"
    grep '^{' "$O/emu8.log" > "$O/emu8.json" && cut -c 1-300 "$O/emu8.json"
fi
if has emu8trace; then
    run trace_emu8 600 rocprofv3 --kernel-trace --stats -d "$O/trace_emu8" -o k -f csv -- python3 bench.py --emulate-shard 8 --steps 40 --warmup 4 --no-cpu --inflight 1 --prof-steps 4 --latency-batches 0
    find "$O/trace_emu8" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_emu8.csv" \;
    head -14 "$O/kernel_stats_emu8.csv" | cut -c 1-160
fi
if has tier5; then
    # configs[4]'s per-GPU shape: the cfg4 rank-0 shard (37 GB) served from a shard file through an
    # HBM cache smaller than the shard (io_uring + O_DIRECT, next-use eviction, prefetch)
    run tier5 1000 python3 -u bench.py $CFG4 --steps 20 --warmup 2 --prof-steps 4 --tier-cache-gib ${TIER_GIB:-24} --tier-call 512 --tier-calls ${TIER_CALLS:-4}
    grep '^{' "$O/tier5.log" > "$O/tier5.json" && python3 -c "import json; d=json.load(open('$O/tier5.json')); print(json.dumps(d.get('tier')))"
fi
if has shardtrace; then
    run trace_cfg4 600 rocprofv3 --kernel-trace --stats -d "$O/trace_cfg4" -o k -f csv -- python3 bench.py $CFG4 --steps 20 --warmup 2 --inflight 1 --latency-batches 0
    find "$O/trace_cfg4" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_cfg4_shard.csv" \;
    head -6 "$O/kernel_stats_cfg4_shard.csv"
fi
echo "profile_round $TAG done"
