# Parity (parity + bounded files) then the 1/8-shard, headline and cfg4-shard bench lines
# (run via gpurun).  usage: bash tools/session_lines.sh <tag> [extra bench args]
set -o pipefail
TAG=$1; shift; X="$*"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bounded.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
line() {  # line <name> <args>
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py --no-cpu "$@" $X > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], 'scan', d['roofline']['scan_ms_per_launch'], 'frac', d['roofline']['frac'])"
}
line shard8 --emulate-shard 8 --inflight 3
line cfg3
line cfg4 --cfg cfg4 --emulate-shard 8 --inflight 3
line shard8b --emulate-shard 8 --inflight 3
