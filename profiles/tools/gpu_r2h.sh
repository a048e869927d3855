#!/bin/bash
# Round-2 HEAD: C2 and C4 bench lines (builder-side evidence beside the driver's C3 line).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config c2 > gpurun_out/bench_c2_h.json 2> gpurun_out/bench_c2_h.err || { tail -20 gpurun_out/bench_c2_h.err; exit 1; }
cat gpurun_out/bench_c2_h.json
timeout -k 10 700 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_h.json 2> gpurun_out/bench_c4_h.err || { tail -20 gpurun_out/bench_c4_h.err; exit 1; }
cat gpurun_out/bench_c4_h.json
