#!/bin/sh
# A/B timing on one box: bench.py (C3 shard, no CPU leg) with each variant library.
for v in "$@"; do
  MT_LIB_PATH=fluidframework_amd/libmtreplay_$v.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
