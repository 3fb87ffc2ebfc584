# the 1/8 shard with the emulated 8-record exchange on its timeline: slots x in-flight depth
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v; mkdir -p $O
i=0
run() {  # run <variant or -> <args...>
  L=$1; shift; i=$((i+1))
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/_variants/$L/libvdb_ivf.so; fi
  timeout -k 10 400 python3 -u bench.py --emulate-shard 8 --emulate-exchange --steps 300 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 "$@" > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$L $*]', d['value'], d['ms_per_step'], 'lat', d['latency_mean_ms'])"
}
run - --inflight 3
run slots4 --inflight 4
run slots6 --inflight 6
run slots6 --inflight 5
unset VDB_IVF_LIB
