#!/bin/bash
# Round 3: the whole -m gpu suite after the growth step, an A/B of the C3 shard replay against
# the round-start library (bench_libs/libmt_base.so, built from cb3d48e), the C5 bench.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3i.log 2>&1; rc=$?
tail -n 5 gpurun_out/pytest_gpu_r3i.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3i_${v}_$i.json 2> gpurun_out/ab_r3i_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3i_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_r3i.json 2> gpurun_out/bench_c5_r3i.err; rc=$?
tail -n 3 gpurun_out/bench_c5_r3i.err
python -c "import json; d=json.load(open('gpurun_out/bench_c5_r3i.json')); print(d['value'], d['summary_decode']['value'], d['end_to_end'])"
exit $rc
