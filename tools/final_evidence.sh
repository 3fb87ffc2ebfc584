#!/bin/bash
# Round-end evidence at the current build (run via gpurun from the repo root): screen tests,
# PMC traffic (headline, mixture, cfg4 shard) stamped with the build id, the headline and
# mixture bench lines, kernel traces, and MFMA-busy counters of the screened scan.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03fin4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_screen.py -q --timeout 300 --timeout-method thread > $O/pytest_screen.log 2>&1 || { tail -5 $O/pytest_screen.log; exit 1; }
tail -1 $O/pytest_screen.log
bash tools/profile_round.sh $(basename $O) traffic,traffic4,bench,trace || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-include-regex "ivf_scan_screen|ivf_coarse|ivf_select_rerank" -d $O/mfma_pmc -o m -f csv \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 > $O/mfma_pmc.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "ivf_scan_screen|ivf_coarse|ivf_select_rerank" \
    -d $O/mfma_trace -o t -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --prof-steps 2 > $O/mfma_trace.log 2>&1 || exit $?
python3 tools/mfma_report.py $O/mfma_pmc $O/mfma_trace $O/mfma.json | tail -12
