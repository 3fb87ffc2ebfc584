# workspace slots x batches in flight at the 1/8 shard (engine variants via VDB_IVF_LIB)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p; mkdir -p $O
i=0
run() {  # run <lib or -> <args...>
  L=$1; shift; i=$((i+1))
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/$L; fi
  timeout -k 10 400 python3 -u bench.py --emulate-shard 8 --steps 300 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 "$@" > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$L $*]', d['value'], d['ms_per_step'], 'lat', d['latency_mean_ms'])"
}
run - --inflight 3
run - --inflight 3 --opt scan_blocks=384
run _variants/slots4/libvdb_ivf.so --inflight 4
run _variants/slots4/libvdb_ivf.so --inflight 4 --opt scan_blocks=384
run _variants/slots6/libvdb_ivf.so --inflight 6
run _variants/slots6/libvdb_ivf.so --inflight 6 --opt scan_blocks=384
run _variants/slots6/libvdb_ivf.so --inflight 3
unset VDB_IVF_LIB
