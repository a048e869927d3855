#!/bin/bash
# Round 3: live-client tests (k_regen's sizing pass) + the Node facade + summaries.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_live_client.py tests/test_js_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3p.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_r3p.log
exit $rc
