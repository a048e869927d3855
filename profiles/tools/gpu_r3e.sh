#!/bin/bash
# Round 3: Node facade (events with ordinals, read-outs, Client.snapshot, flushAsync), event /
# read-out parity, summary loads with MT_DOC_ALIASED (every reference document compared).
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_js_facade.py tests/test_events.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/pytest_r3e.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "snapshot or summaries" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3e_snap.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r3e_snap.log
exit $rc
