#!/bin/bash
# the whole GPU suite on the final build: every file but the large configs, then the large configs
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
T=$(ls tests/test_gpu_*.py | grep -v large_configs)
timeout -k 10 900 python -u -m pytest $T -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_all_but_large.log 2>&1
rc=$?; tail -3 $O/pytest_all_but_large.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_large_configs.py -m gpu -q -rf --timeout 900 --timeout-method thread > $O/pytest_large.log 2>&1
rc=$?; tail -3 $O/pytest_large.log; exit $rc
