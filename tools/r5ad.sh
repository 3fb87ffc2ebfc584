#!/bin/bash
# calibration batch capped by batch_cap (int8 for every item width): the GPU suite without the
# large-config files, then cfg4 with the automatic shadow
set -o pipefail
T=$(ls tests/test_gpu_*.py | grep -v large_configs | tr '\n' ';')
bash tools/r4_gpu.sh r5ad "t:$T@s:cfg4:|inflight=3"
