set -o pipefail
O=gpurun_out/s12; mkdir -p $O
bash tools/trace_ab.sh s12 - mb1024 | grep -i "merge_partials\|plan\|scan_wide" || exit 1
for v in - mb1024; do
  if [ "$v" = "-" ]; then unset VDB_IVF_LIB; n=intree; else export VDB_IVF_LIB=$PWD/_variants/$v/libvdb_ivf.so; n=$v; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench_$n.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_$n.log 2>&1 || exit 1
  unset VDB_IVF_LIB
  for f in bench shard8; do grep '^{' $O/${f}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n $f', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'])"; done
done
