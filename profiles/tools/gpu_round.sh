#!/bin/bash
# Re-entry check on the GPU box: -m gpu suite, default bench (C2), C3 at the 8-GPU per-rank share.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 500 python -u bench.py --config c3 --docs 12500 --no-cpu --steps 1 --warmup 1 > gpurun_out/c3_12500.json 2>gpurun_out/c3_12500.err || { tail -20 gpurun_out/c3_12500.err; exit 1; }
cat gpurun_out/c3_12500.json
