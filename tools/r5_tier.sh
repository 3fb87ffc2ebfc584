#!/bin/bash
# configs[4] shape on the final build: cfg4 rank 0 of 5 (19.3M vectors, 61.65 GB shard file) through
# the screened tier at cache $1 GiB (24 = 0.42 of the lists, 11.5 = 0.2); row cache by size, then
# refilled by a survivor histogram of 4096 other queries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
c=$1
timeout -k 10 1100 python3 -u bench.py --cfg cfg4 --emulate-shard 5 --steps 20 --warmup 2 --no-cpu --latency-batches 0 --prof-steps 3 \
   --tier-cache-gib $c --tier-call 512 --tier-calls 4 --tier-adapt 4096 > $O/tier_$c.log 2>&1 || { tail -30 $O/tier_$c.log; exit 1; }
grep '^{' $O/tier_$c.log > $O/tier_$c.json
python3 -c "
import json; d=json.load(open('$O/tier_$c.json')); t=d['tier']
print('cache', t['cache_gib'], t['cache_fraction_of_lists'], 'QPS', t['value'], 'rows read', t['survivor_rows_per_batch'], 'cached', t['survivor_rows_from_hbm_cache_per_batch'], 'gbps', t['file_read_gbps'], 'parity', t['parity_with_resident_index'])
for v in t.get('variants', []): print('   ', v)
print('resident', d['value'], d['ms_per_step'])"
