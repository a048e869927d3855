#!/bin/bash
# Round 3: page hints in paged zamboni heap entries (bench_libs/libmt_hint.so): parity on
# every tier, C3 12.5k-shard A/B against HEAD (bench_libs/libmt_head.so), C4.
set -u
mkdir -p gpurun_out
MT_LIB_PATH=$PWD/bench_libs/libmt_hint.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_events.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3x.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_r3x.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in head hint; do
    MT_LIB_PATH=$PWD/bench_libs/libmt_$v.so timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3x_${v}_$i.json 2> gpurun_out/ab_r3x_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3x_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d.get('parity',{}).get('replay_equals_generation'))"
  done
done
for v in head hint; do
  MT_LIB_PATH=$PWD/bench_libs/libmt_$v.so timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3x_c4_$v.json 2> gpurun_out/ab_r3x_c4_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3x_c4_$v.json')); print('c4 $v', d['value'], d['ms_per_step'], d.get('parity',{}).get('replay_equals_generation'))"
done
