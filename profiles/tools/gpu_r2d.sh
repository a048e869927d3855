#!/bin/bash
# Round-2 check at HEAD: -m gpu suite, smoke, default bench line, live-client bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_d.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_d.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_d.json 2> gpurun_out/bench_c3_d.err || { tail -20 gpurun_out/bench_c3_d.err; exit 1; }
cat gpurun_out/bench_c3_d.json
timeout -k 10 500 python -u bench.py --config live --steps 3 --warmup 1 > gpurun_out/bench_live_d.json 2> gpurun_out/bench_live_d.err || { tail -20 gpurun_out/bench_live_d.err; exit 1; }
cat gpurun_out/bench_live_d.json
