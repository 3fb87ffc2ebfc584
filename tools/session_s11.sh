set -o pipefail
O=gpurun_out/s11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VDB_IVF_LIB=$PWD/_variants/plan_ts_s2/libvdb_ivf.so timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu --inflight 1 > $O/plan_ts.log 2>&1 || exit 1
grep plan_ts $O/plan_ts.log | tail -3
bash tools/trace_ab.sh s11 - || exit 1
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log > $O/bench.json; cut -c 1-300 $O/bench.json
python3 -c "import json; d=json.load(open(\"$O/bench.json\")); print(\"distinct_lists\", d[\"roofline\"][\"distinct_lists_per_batch\"], \"scan\", d[\"roofline\"][\"scan_ms_per_launch\"])"
