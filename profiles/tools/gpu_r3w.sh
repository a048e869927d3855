#!/bin/bash
# Round 3: C4's tight tier with 32-bit overlap masks and a packed table (narrow + packed,
# bench_libs/libmt_narrow4.so, MT_BENCH_C4_NARROW=1): fast-path parity at the bench's
# capacities, then C4 A/B against HEAD (bench_libs/libmt_head.so) and a C3 shard check.
set -u
mkdir -p gpurun_out
MT_LIB_PATH=$PWD/bench_libs/libmt_narrow4.so MT_BENCH_C4_NARROW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fast_path or full_streams or long_documents or grow" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3w.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_r3w.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  MT_LIB_PATH=$PWD/bench_libs/libmt_head.so timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3w_c4_head_$i.json 2> gpurun_out/ab_r3w_c4_head_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3w_c4_head_$i.json')); print('c4 head', d['value'], d['ms_per_step'], d['roofline']['paged_peaks'], d['parity']['replay_equals_generation'])"
  MT_LIB_PATH=$PWD/bench_libs/libmt_narrow4.so MT_BENCH_C4_NARROW=1 timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3w_c4_n4_$i.json 2> gpurun_out/ab_r3w_c4_n4_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3w_c4_n4_$i.json')); print('c4 narrow4', d['value'], d['ms_per_step'], d['roofline']['paged_peaks'], d['parity']['replay_equals_generation'])"
done
MT_LIB_PATH=$PWD/bench_libs/libmt_narrow4.so MT_BENCH_C4_NARROW=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/ab_r3w_c4_n4_oracle.json 2> gpurun_out/ab_r3w_c4_n4_oracle.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab_r3w_c4_n4_oracle.json')); print('c4 narrow4 oracle sample', d['parity'])"
for v in head narrow4; do
  MT_LIB_PATH=$PWD/bench_libs/libmt_$v.so timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3w_c3_$v.json 2> gpurun_out/ab_r3w_c3_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3w_c3_$v.json')); print('c3 $v', d['ms_per_step'])"
done
