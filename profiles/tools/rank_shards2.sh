#!/bin/bash
# every rank's C3 shard of the 8-GPU job on one GPU at the default (tight) paged capacities:
# peaks vs capacities (a fallback would show the loose capacities) and the per-shard rate
set -u
mkdir -p gpurun_out/shards
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --shard $r > gpurun_out/shards/rank_$r.json 2>gpurun_out/shards/rank_$r.err || { echo "rank $r failed"; tail -3 gpurun_out/shards/rank_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/shards/rank_$r.json')); print('rank $r', round(d['value']/1e6,2), d['roofline']['paged_peaks'], d['roofline']['paged_caps'], d['parity']['replay_equals_generation'])"
done
