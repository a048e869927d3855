#!/bin/bash
# Round 3: growth tests with the per-region kernels, C3 shard A/B against the round-start
# library, the C5 bench (end-to-end leg with the tail client remap).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "grow or capacity" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3l_grow.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_r3l_grow.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3l_${v}_$i.json 2> gpurun_out/ab_r3l_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3l_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_r3l.json 2> gpurun_out/bench_c5_r3l.err; rc=$?
tail -n 3 gpurun_out/bench_c5_r3l.err
python -c "import json; d=json.load(open('gpurun_out/bench_c5_r3l.json')); print(d['value'], d['summary_decode']['value'], d['end_to_end'])"
exit $rc
