#!/bin/bash
# -m gpu suite (incl. maintenance-event parity), then a short C3 bench (no CPU leg).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu5.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu5.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_maint.json 2> gpurun_out/bench_maint.err || { tail -20 gpurun_out/bench_maint.err; exit 1; }
cat gpurun_out/bench_maint.json
