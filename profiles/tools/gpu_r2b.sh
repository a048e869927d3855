#!/bin/bash
# Round-2 re-entry check at HEAD: the -m gpu suite, smoke, then the default bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_b.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_b.json 2> gpurun_out/bench_c3_b.err || { tail -20 gpurun_out/bench_c3_b.err; exit 1; }
cat gpurun_out/bench_c3_b.json
