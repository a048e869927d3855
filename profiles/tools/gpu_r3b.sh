#!/bin/bash
# Round 3: segment ordinals / event parity / read-outs on the GPU, then the whole -m gpu
# suite, then an A/B of the replay fast path (C3 12.5k shard) against the library built
# from the previous commit (bench_libs/libmt_base.so).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_events.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b_events.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/pytest_r3b_events.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3b.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_r3b.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3b_${v}_$i.json 2> gpurun_out/ab_r3b_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3b_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
