#!/bin/bash
# GPU sessions (run via gpurun from the repo root), one parametrised recipe for every
# measurement of round 6 (profiles/INDEX.md names the tag and steps behind each record):
#   bash tools/session.sh <tag> <step,step,...>
#   smoke     __graft_entry__.smoke()
#   multi     the two-rank rehearsal of the N-rank path on one GPU (bench.py --gpus 2)
#   grpc      the gRPC front end under load (tools/grpc_load.py)
#   sweep     tools/knob_sweep.py $SWEEP_WL (default "s8 cfg3") over $SWEEP_SETS (engine option sets)
#   trace8    the 1/8 shard at 3 in flight under a kernel trace, its timeline (tools/timeline.py)
#   prof8     rocprofv3 kernel trace of the 1/8-shard rehearsal (headline index, rank 0 of 8), one in flight
#   prof3     the same for the headline, one and two in flight
#   tier      configs[4] shape: cfg4 rank 0 of 5 as a shard file through the screened tier at
#             TIER_GIB (default 11.5 = 0.2 of the lists), two-pass vs one-pass re-check, refill
#   probe     the disk's random-read ceiling (tools/rand_read_probe.cpp)
#   ranks3    every rank of the 8-GPU headline, a process each, emulated 8-record exchange
#   ranks4    the same for configs[3]
#   tests     pytest -m gpu (PYTEST_K: -k filter)
#   bench     the default bench line
set -o pipefail
TAG=$1; STEPS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
run() {  # run <name> <seconds> <cmd...>: stop at the first failure
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
if has tests; then
    run pytest 1100 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
    tail -3 "$O/pytest.log"
fi
if has smoke; then
    run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
    tail -2 "$O/smoke.log"
fi
if has multi; then
    run multi 600 python -u bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --prof-steps 4
    grep '^{' "$O/multi.log" > "$O/multi.json"
    cut -c 1-400 "$O/multi.json"
fi
if has grpc; then
    run grpc 600 python -u tools/grpc_load.py
    grep '^{' "$O/grpc.log" > "$O/grpc.json"
    cat "$O/grpc.json"
fi
if has prof8; then
    run prof8 400 rocprofv3 --kernel-trace --stats -d "$O/prof8" -o k -f csv -- python3 bench.py --emulate-shard 8 --inflight 1 --steps 30 --warmup 3 --no-cpu --latency-batches 0 --prof-steps 5
    find "$O/prof8" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_emu8.csv" \;
    cut -d, -f1-4 "$O/kernel_stats_emu8.csv" | cut -c1-150 | head -24
fi
if has trace8; then
    # the 1/8 shard at 3 in flight under a kernel trace: the timed region's timeline (tools/timeline.py)
    run trace8 400 rocprofv3 --kernel-trace -d "$O/trace8" -o k -f csv -- python3 bench.py --emulate-shard 8 --inflight 3 --steps 100 --warmup 5 --no-cpu --latency-batches 0 --prof-steps 2
    python3 tools/timeline.py "$(find "$O/trace8" -name '*kernel_trace.csv' | head -1)" 100 > "$O/timeline8.json" && cut -c1-1500 "$O/timeline8.json"
fi
if has prof3; then
    for inf in 1 2; do
        run prof3_$inf 400 rocprofv3 --kernel-trace --stats -d "$O/prof3_$inf" -o k -f csv -- python3 bench.py --inflight $inf --steps 30 --warmup 3 --no-cpu --latency-batches 0 --prof-steps 5
        find "$O/prof3_$inf" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_inflight$inf.csv" \;
        cut -d, -f1-4 "$O/kernel_stats_inflight$inf.csv" | cut -c1-150 | head -16
    done
fi
if has probe; then
    g++ -O2 -std=c++17 -o /tmp/rand_read_probe tools/rand_read_probe.cpp || exit 1
    run probe 300 /tmp/rand_read_probe /tmp 24 256 5
    cat "$O/probe.log"
fi
if has tier; then
    c=${TIER_GIB:-11.5}
    run tier 1150 python3 -u bench.py --cfg cfg4 --emulate-shard 5 --steps 20 --warmup 2 --no-cpu --latency-batches 0 --prof-steps 3 \
        --tier-cache-gib $c --tier-call 512 --tier-calls 4 --tier-variant screen_recheck2=0 --tier-adapt 4096
    grep '^{' "$O/tier.log" > "$O/tier.json"
    python3 -c "
import json; d=json.load(open('$O/tier.json')); t=d['tier']
print('cache', t['cache_gib'], t['cache_fraction_of_lists'], 'QPS', t['value'], 'rows read', t['survivor_rows_per_batch'], 'cached', t['survivor_rows_from_hbm_cache_per_batch'], 'amp', t.get('read_amplification'), 'gbps', t['file_read_gbps'], 'parity', t['parity_with_resident_index'])
for v in t.get('variants', []): print('   ', v)
print('resident', d['value'], d['ms_per_step'])"
fi
if has ranks3; then
    run ranks3 900 python -u bench.py --cfg cfg3 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/ranks3.log" > "$O/ranks3.json"
    cut -c 1-600 "$O/ranks3.json"
fi
if has ranks3q; then
    # the same with 4 workspace slots (a _variants/slots4 build), 4 batches in flight and 8 hardware
    # queues per process (4 in-flight streams + the communicator's each on a queue of their own)
    run ranks3q 900 env VDB_IVF_LIB=$R/_variants/slots4/libvdb_ivf.so GPU_MAX_HW_QUEUES=8 python -u bench.py --cfg cfg3 --emulate-rank all --emulate-shard 8 --inflight 4 --no-cpu
    grep '^{' "$O/ranks3q.log" > "$O/ranks3q.json"
    cut -c 1-600 "$O/ranks3q.json"
fi
if has ranks4; then
    run ranks4 1100 python -u bench.py --cfg cfg4 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/ranks4.log" > "$O/ranks4.json"
    cut -c 1-600 "$O/ranks4.json"
fi
if has sweep; then
    # one build, several option sets: tools/knob_sweep.py $SWEEP_WL $SWEEP_SETS
    for wl in ${SWEEP_WL:-s8 cfg3}; do
        run sweep_$wl 900 python -u tools/knob_sweep.py $wl $SWEEP_SETS
        grep '^{' "$O/sweep_$wl.log" | cut -c1-330
    done
fi
if has sweepq; then
    # the sweep on the 4-slot build (_variants/slots4) with 8 hardware queues per process
    for wl in ${SWEEP_WL:-s8 cfg3}; do
        run sweepq_$wl 900 env VDB_IVF_LIB=$R/_variants/slots4/libvdb_ivf.so GPU_MAX_HW_QUEUES=8 python -u tools/knob_sweep.py $wl $SWEEP_SETS
        grep '^{' "$O/sweepq_$wl.log" | cut -c1-330
    done
fi
if has sweepv; then
    # the sweep on an A/B library: _variants/$VARIANT (tools/build_*variant.sh)
    for wl in ${SWEEP_WL:-s8 cfg3}; do
        run sweepv_$wl 900 env VDB_IVF_LIB=$R/_variants/$VARIANT/libvdb_ivf.so python -u tools/knob_sweep.py $wl $SWEEP_SETS
        grep '^{' "$O/sweepv_$wl.log" | cut -c1-330
    done
fi
if has ranks3v; then
    run ranks3v 900 env VDB_IVF_LIB=$R/_variants/$VARIANT/libvdb_ivf.so python -u bench.py --cfg cfg3 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/ranks3v.log" > "$O/ranks3v.json"
    cut -c 1-600 "$O/ranks3v.json"
fi
if has bench; then
    run bench 600 python -u bench.py ${BENCH_ARGS}
    grep '^{' "$O/bench.log" > "$O/bench.json"
    cut -c 1-400 "$O/bench.json"
fi
echo "session $TAG done"
