#!/bin/bash
# Round 3: live documents staged in LDS (TierLiveLdsT, bench_libs/libmt_livelds.so): the live
# tests on the HBM tier and with 64 / 192-segment LDS tiers, then the live bench line
# (HEAD library, HBM tier) vs the variant (HBM tier; LDS tier 192 / 256 segments).
set -u
mkdir -p gpurun_out
export MT_LIB_PATH=$PWD/bench_libs/libmt_livelds.so
timeout -k 10 600 python -u -m pytest tests/test_live_client.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3v.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_r3v.log | tail -20
[ $rc -eq 0 ] || exit $rc
for v in head livelds; do
  MT_LIB_PATH=$PWD/bench_libs/libmt_$v.so timeout -k 10 300 python -u bench.py --config live --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_r3v_$v.json 2> gpurun_out/ab_r3v_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3v_$v.json')); print('$v hbm', d['value'], d['ms_per_step'], d['parity'])"
done
for c in 192 384 768; do
  timeout -k 10 300 python -u bench.py --config live --steps 5 --warmup 1 --lds-cap $c > gpurun_out/ab_r3v_lds$c.json 2> gpurun_out/ab_r3v_lds$c.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_r3v_lds$c.json')); print('livelds lds$c', d['value'], d['ms_per_step'], d['parity'], d['cpu_baseline']['value'])"
done
