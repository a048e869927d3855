#!/bin/bash
# Round 3: lazy unsettled-table invalidation (bench_libs/libmt_lazy.so): parity on the paged
# tiers, C3 12.5k-shard A/B against the round-start library, C4 bench.
set -u
mkdir -p gpurun_out
export MT_LIB_PATH=$PWD/bench_libs/libmt_lazy.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_events.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3q.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_r3q.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base lazy; do
    lib=$PWD/bench_libs/libmt_$v.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3q_${v}_$i.json 2> gpurun_out/ab_r3q_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3q_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['paged_peaks'])"
  done
done
timeout -k 10 600 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_r3q.json 2> gpurun_out/bench_c4_r3q.err || { tail -n 5 gpurun_out/bench_c4_r3q.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4_r3q.json')); print('c4', d['value'], d['ms_per_step'], d['roofline'].get('paged_peaks'), d['parity'])"
