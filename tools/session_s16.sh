set -o pipefail
O=$PWD/gpurun_out/s16; mkdir -p $O
for v in - pool1 -; do
  if [ "$v" = "-" ]; then unset VDB_IVF_LIB; n=head; else export VDB_IVF_LIB=$PWD/_variants/$v/libvdb_ivf.so; n=$v; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_$n.log 2>&1 || { tail -5 $O/shard8_$n.log; exit 1; }
  unset VDB_IVF_LIB
  grep '^{' $O/shard8_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n shard8', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log > $O/bench.json; cut -c 1-330 $O/bench.json
