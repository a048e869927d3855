#!/bin/bash
# Round-2: C5 bench line with the native summary decoder's host rate (summary_decode).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config c5 > gpurun_out/bench_c5_e.json 2> gpurun_out/bench_c5_e.err || { tail -20 gpurun_out/bench_c5_e.err; exit 1; }
cat gpurun_out/bench_c5_e.json
