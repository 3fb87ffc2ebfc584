set -o pipefail
O=gpurun_out/st; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_bounded.sh st8 "--emulate-shard 8 --inflight 3" "-" || exit 1
bash tools/ab_bounded.sh st3 "" "-" || exit 1
bash tools/ab_bounded.sh st4 "--cfg cfg4 --emulate-shard 8 --inflight 3" "-" || exit 1
