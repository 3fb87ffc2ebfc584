# Per-GPU work of the 8-GPU headline: rank 0 of an 8-way LPT shard of cfg3 (no all-gather),
# bench line + kernel trace (run via gpurun).
set -o pipefail
O=gpurun_out/${1:-s8}; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --emulate-shard 8 --no-cpu --inflight 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json && cut -c 1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o k -f csv -- python3 bench.py --emulate-shard 8 --no-cpu --inflight 3 --steps 40 --warmup 4 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace1 -o k -f csv -- python3 bench.py --emulate-shard 8 --no-cpu --inflight 1 --steps 40 --warmup 4 > $O/trace1.log 2>&1 || { tail -20 $O/trace1.log; exit 1; }
find $O/trace1 -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_one_in_flight.csv \;
