set -o pipefail
O=gpurun_out/s13; mkdir -p $O
for v in - fq0now k0c2 -; do
  if [ "$v" = "-" ]; then unset VDB_IVF_LIB; n=intree; else export VDB_IVF_LIB=$PWD/_variants/$v/libvdb_ivf.so; n=$v; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --emulate-shard 8 --inflight 3 > $O/shard8_$n.log 2>&1 || exit 1
  unset VDB_IVF_LIB
  grep '^{' $O/shard8_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n shard8', d['value'], d['ms_per_step'], d['p99_ms_one_in_flight'], d['roofline']['scan_ms_per_launch'], d['roofline']['search_ms_per_batch'])"
done
