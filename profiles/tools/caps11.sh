#!/bin/bash
# Paged LDS capacities: 16.0 KB (10 documents per CU) vs 14.8 KB (11 per CU) on C3 shards.
set -u
mkdir -p gpurun_out/caps11
for sh in 0 5; do
  for caps in 208,240,224 192,216,208; do
    timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 --shard $sh --page-caps $caps \
        > gpurun_out/caps11/s${sh}_${caps}.json 2> gpurun_out/caps11/s${sh}_${caps}.err || { tail -5 gpurun_out/caps11/s${sh}_${caps}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,2), d['ms_per_step'], d['roofline'].get('paged_caps'), d['roofline'].get('paged_peaks'))" gpurun_out/caps11/s${sh}_${caps}.json $sh $caps
  done
done
