#!/bin/bash
# Live-client path: the -m gpu tests of tests/test_live_client.py and the Node facade's live test.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_live_client.py tests/test_js_facade.py -k "live" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_live.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_live.log | head -40
exit $rc
