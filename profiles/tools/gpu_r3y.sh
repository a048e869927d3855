#!/bin/bash
# Round 3: the live path against the C restatement's participant replay (checksums), and the
# live bench line with its new CPU baseline.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_live_client.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r3y.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/pytest_r3y.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config live --steps 5 --warmup 1 > gpurun_out/bench_live_r3y.json 2> gpurun_out/bench_live_r3y.err || exit 1
cat gpurun_out/bench_live_r3y.json
