#!/bin/bash
# Round-2: native summary decoder on the GPU paths (Python load_summaries, Node loadSnapshots).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_facade.py tests/test_snapdec.py -x -v --timeout 300 --timeout-method thread -k "summar or snapshot or snapdec" > gpurun_out/pytest_snapdec.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_snapdec.log | tail -15
exit $rc
