#!/bin/bash
# every rank of the 8-GPU headline and of the 8-GPU configs[3] job, a process each, emulated exchange
set -o pipefail
bash tools/r5_ranks.sh || exit $?
bash tools/r5_ranks4.sh
