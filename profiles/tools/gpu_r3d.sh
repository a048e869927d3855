#!/bin/bash
# Round 3: the Node facade's SharedSegmentSequence surface on the GPU (events with ordinals,
# read-outs, Client.snapshot, flushAsync) and the event / read-out parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_js_facade.py tests/test_events.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/pytest_r3d.log | tail -40
exit $rc
