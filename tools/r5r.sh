# collect variants (k-steps in flight of the int8 shadow, threshold re-read interval): bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5r; mkdir -p $O
i=0
run() {  # run <lib or -> <args...>
  L=$1; shift; i=$((i+1))
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/_variants/$L/libvdb_ivf.so; fi
  timeout -k 10 400 python3 -u bench.py --steps 300 --warmup 20 --no-cpu --latency-batches 0 --prof-steps 10 "$@" > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$L $*]', d['value'], d['ms_per_step'], 'collect', r['kernel_ms_per_launch'])"
}
for L in - kd6 te16 kd6te; do
  X=""; [ "$L" = te16 -o "$L" = kd6te ] && X="--opt screen_thr_every=4"
  run $L --emulate-shard 8 --inflight 3 $X
  run $L $X
done
unset VDB_IVF_LIB
