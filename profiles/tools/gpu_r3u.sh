#!/bin/bash
# Round 3: C4 with its packed tight tier fixed at compile time (HEAD) vs without
# (bench_libs/libmt_fixed.so), interleaved; fast-path parity at the C4 capacities first.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_streams" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3u.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_r3u.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in fixed head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = fixed ] && lib=$PWD/bench_libs/libmt_fixed.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3u_${v}_$i.json 2> gpurun_out/ab_r3u_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3u_${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity']['replay_equals_generation'])"
  done
done
