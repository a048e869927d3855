#!/bin/bash
# Round-2 evidence: default bench (C3 shard) with the CPU baseline, the rocprofv3 trace/PMC
# passes for it, then one run at the full 100k-document job on one GPU (no CPU leg).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json || exit 1
timeout -k 10 400 python -u bench.py --docs 100000 --no-cpu --steps 2 --warmup 1 > gpurun_out/bench_c3_100k.json 2> gpurun_out/bench_c3_100k.err || { tail -20 gpurun_out/bench_c3_100k.err; exit 1; }
cat gpurun_out/bench_c3_100k.json
