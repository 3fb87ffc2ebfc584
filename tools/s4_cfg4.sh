set -o pipefail
O=gpurun_out/s4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sharded_build or two_shards" -x -v --timeout 120 --timeout-method thread > $O/pt.log 2>&1; rc=$?; tail -4 $O/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --cfg cfg4 --emulate-shard 8 --no-cpu --inflight 3 > $O/cfg4.log 2>&1; rc=$?; tail -3 $O/cfg4.log | cut -c1-1500; exit $rc
