#!/bin/bash
# Round-4 GPU session helper (run through gpurun from the repo root):
#   bash tools/r4_gpu.sh <tag> <step>[@<step>...]
# steps: t:<pytest args, ';'-separated files> | s:<workload>:<opt sets separated by '|'> | b:<bench args>
#        p:<workload>:<opt sets> (the sweep under rocprofv3 --kernel-trace --stats)
#        m:<counters ';'-separated>:<workload>:<opt sets> (one rocprofv3 --pmc pass over the sweep)
#        q:<bench args> (bench.py under rocprofv3 --kernel-trace --stats)
# Each step runs under its own time limit; a crash (abort, segfault, time limit) ends the
# session, a failed assertion does not (the next steps still measure).
set -o pipefail
TAG=$1
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
IFS='@' read -ra STEPS <<< "$2"
for st in "${STEPS[@]}"; do
    i=$((i + 1))
    kind=${st%%:*}
    arg=${st#*:}
    case $kind in
        t) timeout -k 10 900 python -u -m pytest ${arg//;/ } -m gpu -q -rf --timeout 300 --timeout-method thread > "$O/$i.pytest.log" 2>&1
           rc=$?; tail -15 "$O/$i.pytest.log" ;;
        s) wl=${arg%%:*}; sets=${arg#*:}
           IFS='|' read -ra SETS <<< "$sets"
           timeout -k 10 900 python -u tools/knob_sweep.py "$wl" "${SETS[@]}" > "$O/$i.sweep_$wl.log" 2>&1
           rc=$?; grep '^{' "$O/$i.sweep_$wl.log" ;;
        p) wl=${arg%%:*}; sets=${arg#*:}
           IFS='|' read -ra SETS <<< "$sets"
           timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof$i" -o run -- python3 -u tools/knob_sweep.py "$wl" "${SETS[@]}" > "$O/$i.prof_$wl.log" 2>&1
           rc=$?; grep '^{' "$O/$i.prof_$wl.log"; f=$(find "$O/prof$i" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -25 ;;
        m) cnt=${arg%%:*}; rest=${arg#*:}; wl=${rest%%:*}; sets=${rest#*:}
           IFS='|' read -ra SETS <<< "$sets"
           timeout -s KILL 600 rocprofv3 --pmc ${cnt//;/ } --kernel-include-regex "ivf_screen_collect|ivf_scan_" -d "$O/pmc$i" -o run -f csv -- python3 -u tools/knob_sweep.py "$wl" "${SETS[@]}" > "$O/$i.pmc_$wl.log" 2>&1
           rc=$?; grep '^{' "$O/$i.pmc_$wl.log"; find "$O/pmc$i" -name '*counter_collection.csv' | head -1 ;;
        q) timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof$i" -o run -- python3 -u bench.py ${arg//;/ } > "$O/$i.qbench.log" 2>&1
           rc=$?; grep '^{' "$O/$i.qbench.log" | cut -c 1-1500; find "$O/prof$i" -name '*kernel_stats.csv' | head -3 ;;
        b) timeout -k 10 900 python -u bench.py ${arg//;/ } > "$O/$i.bench.log" 2>&1
           rc=$?; grep '^{' "$O/$i.bench.log" | cut -c 1-1500 ;;
    esac
    echo "[step $i $kind] rc=$rc"
    case $rc in 0|1) ;; *) tail -30 "$O/$i."*.log; exit $rc ;; esac
done
