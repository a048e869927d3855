#!/bin/bash
# Round 3: the C3 tight tier with compile-time capacities (bench_libs/libmt_fixed.so):
# parity at the bench's capacities, C3 12.5k-shard A/B against the round-start library.
set -u
mkdir -p gpurun_out
MT_LIB_PATH=$PWD/bench_libs/libmt_fixed.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_streams or long_documents or sliced" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3r.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_r3r.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base fixed; do
    MT_LIB_PATH=$PWD/bench_libs/libmt_$v.so timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3r_${v}_$i.json 2> gpurun_out/ab_r3r_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3r_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
