# Round-end evidence, part A (run via gpurun): GPU suite + smoke, plan phase stamps, then
# profile_round's traffic / bench / trace steps.
set -o pipefail
T=${1:-r02final}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
if [ -f _variants/plan_ts/libvdb_ivf.so ]; then
  VDB_IVF_LIB=$PWD/_variants/plan_ts/libvdb_ivf.so timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu --inflight 1 > $O/plan_ts.log 2>&1 || exit 1
  grep plan_ts $O/plan_ts.log | tail -4
fi
bash tools/profile_round.sh $T traffic,traffic4,bench,trace
