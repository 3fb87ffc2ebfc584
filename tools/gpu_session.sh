#!/bin/bash
# One GPU-box session (run via gpurun from the repo root): parity tests, the default
# bench line, the kernel-trace summary of the bench command, PMC passes.
#   usage: bash tools/gpu_session.sh <tag> [steps, comma-separated:
#          tests,smoke,bench,multi,ranks3,ranks4,grpc,prof,pmc]  [extra bench args...]
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
if has ranks3; then
    # every rank's shard of the 8-GPU headline (LPT plan), timed in turn: per-rank balance
    run ranks3 900 python -u bench.py --cfg cfg3 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/ranks3.log" > "$O/ranks3.json"
    cut -c 1-600 "$O/ranks3.json"
fi
if has ranks4; then
    run ranks4 1100 python -u bench.py --cfg cfg4 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/ranks4.log" > "$O/ranks4.json"
    cut -c 1-600 "$O/ranks4.json"
fi
if has ranks3w; then
    run ranks3w 900 python -u bench.py --cfg cfg3 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu --plan weighted
    grep '^{' "$O/ranks3w.log" > "$O/ranks3w.json"
    cut -c 1-300 "$O/ranks3w.json"
fi
if has ranks4w; then
    run ranks4w 1100 python -u bench.py --cfg cfg4 --emulate-rank all --emulate-shard 8 --inflight 3 --no-cpu --plan weighted
    grep '^{' "$O/ranks4w.log" > "$O/ranks4w.json"
    cut -c 1-300 "$O/ranks4w.json"
fi
if has emu8; then
    # rank 0 of 8 cut from the whole headline index by set_shard (round 2's rehearsal line)
    run emu8 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu
    grep '^{' "$O/emu8.log" > "$O/emu8.json"
    cut -c 1-300 "$O/emu8.json"
fi
if has emu8ab; then
    # A/B of one engine option on the 1/8-shard rehearsal line, same box: $AB_OPT=0 vs default
    run emu8a 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu --opt "$AB_OPT=0"
    run emu8b 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu
    run emu8c 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu --opt "$AB_OPT=0"
    run emu8d 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu
    for x in a b c d; do grep '^{' "$O/emu8$x.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$x', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], r['scan_ms_per_launch'], r['search_ms_per_batch'], d['engine_options'])"; done
fi
if has diag4; then
    # cfg4 shard scan under result-invalidating diagnostic builds (_variants/, tools/build_variant.sh):
    # where the scan's time goes (LDS query reads, list reads)
    run diag4_base 600 python -u tools/knob_sweep.py cfg4 ""
    for v in ${DIAG_VARIANTS:-nolds nomem nolds_nomem}; do
        export VDB_IVF_LIB=$R/_variants/$v/libvdb_ivf.so
        run diag4_$v 600 python -u tools/knob_sweep.py cfg4 ""
        unset VDB_IVF_LIB
    done
    for f in "$O"/diag4_*.log; do echo "$(basename $f) $(grep '^{' $f | tail -1)"; done
fi
if has sweep; then
    # one build, several option sets: tools/knob_sweep.py $SWEEP_WL $SWEEP_SETS (scan ms, wall ms per batch)
    for wl in ${SWEEP_WL:-cfg3}; do
        run sweep_$wl 900 python -u tools/knob_sweep.py $wl $SWEEP_SETS
        grep '^{' "$O/sweep_$wl.log"
    done
fi
if has libab; then
    # A/B of two libraries on the same box: the in-tree build vs _variants/$AB_LIB (tools/build_variant.sh),
    # knob_sweep timing (scan ms, wall ms per batch) per workload, alternating A B A B
    for wl in ${AB_WL:-cfg3}; do
        for rep in 1 2; do
            run ab_${wl}_A$rep 900 python -u tools/knob_sweep.py $wl ""
            export VDB_IVF_LIB=$R/_variants/$AB_LIB/libvdb_ivf.so
            run ab_${wl}_B$rep 900 python -u tools/knob_sweep.py $wl ""
            unset VDB_IVF_LIB
            [ "$wl" = cfg4 ] && break
        done
    done
    for f in "$O"/ab_*.log; do echo "$(basename $f .log) $(grep '^{' $f | tail -1 | cut -c1-160)"; done
fi
if has swin; then
    # scan_window A/B at 3 batches in flight (throughput, p99, mean latency): 1/8 shard and cfg4 shard
    run swin_a 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu
    run swin_b 600 python -u bench.py --emulate-shard 8 --inflight 3 --no-cpu --opt scan_window=2
    run swin_c 900 python -u bench.py --cfg cfg4 --emulate-shard 8 --inflight 3 --no-cpu --steps 60 --prof-steps 10
    run swin_d 900 python -u bench.py --cfg cfg4 --emulate-shard 8 --inflight 3 --no-cpu --steps 60 --prof-steps 10 --opt scan_window=2
    for x in a b c d; do grep '^{' "$O/swin_$x.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$x', d['config']['workload'], d['value'], d['ms_per_step'], 'p99', d['p99_ms'], 'mean', d['latency_mean_ms'], d['engine_options'])"; done
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
