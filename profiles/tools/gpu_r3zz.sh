#!/bin/bash
# Round 3 final HEAD check (LDS-staged live tier opt-in): -m gpu suite, smoke, default bench
# line, live line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3zz.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_gpu_r3zz.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_r3zz.json 2> gpurun_out/bench_c3_r3zz.err || { tail -20 gpurun_out/bench_c3_r3zz.err; exit 1; }
cat gpurun_out/bench_c3_r3zz.json
timeout -k 10 300 python -u bench.py --config live --steps 5 --warmup 1 > gpurun_out/bench_live_r3zz.json 2> gpurun_out/bench_live_r3zz.err || exit 1
cat gpurun_out/bench_live_r3zz.json
