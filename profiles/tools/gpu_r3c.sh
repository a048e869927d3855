#!/bin/bash
# A/B of the replay fast path (C3 12.5k shard, default capacities) between the library built
# from an earlier commit (bench_libs/libmt_base.so) and HEAD's, interleaved on one box.
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3c_${v}_$i.json 2> gpurun_out/ab_r3c_${v}_$i.err || { tail -5 gpurun_out/ab_r3c_${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_r3c_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
