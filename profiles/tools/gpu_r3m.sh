#!/bin/bash
# Round 3: packed tight tier (C4: 12-byte unsettled-table entries, 3 documents per CU) --
# parity on the tight / narrow / grow tiers, C4 bench, C3 shard A/B vs the round-start
# library, then the C5 slice probe.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tight or narrow or grow or capacity or full_streams" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3m.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_r3m.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_r3m.json 2> gpurun_out/bench_c4_r3m.err || { tail -n 5 gpurun_out/bench_c4_r3m.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4_r3m.json')); print('c4', d['value'], d['ms_per_step'], d['roofline'].get('paged_peaks'), d.get('cpu_baseline',{}) and d['cpu_baseline'].get('value'), d['parity'])"
for i in 1 2; do
  for v in base head; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3m_${v}_$i.json 2> gpurun_out/ab_r3m_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3m_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 300 python -u tools/probe_c5_slices.py > gpurun_out/probe_c5_r3m.txt 2>&1; tail -n 12 gpurun_out/probe_c5_r3m.txt
