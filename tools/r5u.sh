# configs[4] shape: cfg4 rank 0 of 5 (19.3M vectors, 61.65 GB shard file) through the screened tier
# at cache fractions 0.42 (24 GiB) and 0.2 (11.5 GiB); row cache by size, then by probe census
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5u; mkdir -p $O
for c in 24 11.5; do
  timeout -k 10 1100 python3 -u bench.py --cfg cfg4 --emulate-shard 5 --steps 20 --warmup 2 --no-cpu --latency-batches 0 --prof-steps 3 \
     --tier-cache-gib $c --tier-call 512 --tier-calls 4 --tier-adapt 4096 > $O/tier_$c.log 2>&1 || { tail -30 $O/tier_$c.log; exit 1; }
  grep '^{' $O/tier_$c.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); t=d['tier']
print('cache', t['cache_gib'], t['cache_fraction_of_lists'], 'QPS', t['value'], 'rows read', t['survivor_rows_per_batch'], 'cached', t['survivor_rows_from_hbm_cache_per_batch'], 'gbps', t['file_read_gbps'], 'parity', t['parity_with_resident_index'])
for v in t.get('variants', []): print('   ', v)
print('resident', d['value'], d['ms_per_step'])"
done
