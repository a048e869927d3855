#!/bin/bash
# Round 3 HEAD check after the participant restatement: -m gpu suite, smoke (which checks
# against the oracle), the default bench line (its CPU baseline and parity sample are the
# oracle's).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3z.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_gpu_r3z.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_r3z.json 2> gpurun_out/bench_c3_r3z.err || { tail -20 gpurun_out/bench_c3_r3z.err; exit 1; }
cat gpurun_out/bench_c3_r3z.json
