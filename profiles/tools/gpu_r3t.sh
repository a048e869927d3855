#!/bin/bash
# Round 3: the fast-path parity test (no delta log, bench capacities: the compile-time C3
# tight tier) and the bench-capacity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "full_streams or long_documents" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3t.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_r3t.log | tail -8
exit $rc
