#!/bin/bash
# Default bench (C3 shard) with the CPU baseline, then the rocprofv3 evidence for it.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json
