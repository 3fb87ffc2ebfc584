# cfg4 rank 0 of 8: the 32-query collect at 2 workgroups per CU (variants)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5w; mkdir -p $O
i=0
for L in w2o2k4 w2o2k8; do
  i=$((i+1))
  if [ "$L" = "-" ]; then unset VDB_IVF_LIB; else export VDB_IVF_LIB=$PWD/_variants/$L/libvdb_ivf.so; fi
  timeout -k 10 700 python3 -u tools/knob_sweep.py cfg4 "scan_blocks=512" > $O/s$i.log 2>&1 || { tail -20 $O/s$i.log; exit 1; }
  grep '^{' $O/s$i.log | sed "s/^/[$L] /" | cut -c1-330
done
unset VDB_IVF_LIB
