set -o pipefail
O=gpurun_out/pb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bounded.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_bounded.sh pb4 "--cfg cfg4 --emulate-shard 8 --inflight 3" "-" || exit 1
bash tools/ab_bounded.sh pb3 "" "-" || exit 1
bash tools/shard8_trace.sh s8
