set -o pipefail
O=gpurun_out/s9; mkdir -p $O
for v in plan_ts plan_ts_new; do
  VDB_IVF_LIB=$PWD/_variants/$v/libvdb_ivf.so timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu --inflight 1 > $O/$v.log 2>&1 || exit 1
  grep plan_ts $O/$v.log | tail -3 | sed "s/^/$v /"
done
timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --prof-steps 4 > $O/multi.log 2>&1 || { tail -20 $O/multi.log; exit 1; }
grep '^{' $O/multi.log > $O/multi.json; cut -c 1-400 $O/multi.json
timeout -k 10 400 python3 -u tools/knob_sweep.py cfg4 "" "wide_group=32" > $O/cfg4_wg.jsonl 2>$O/cfg4_wg.err || exit 1
cat $O/cfg4_wg.jsonl
