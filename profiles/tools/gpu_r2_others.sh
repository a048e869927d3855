#!/bin/bash
# Round-2 refresh of the non-default configurations: C2 (with CPU baseline), C4 and C5 bench
# lines, then the rocprofv3 trace + PMC passes for C4.
set -u
mkdir -p gpurun_out
for c in c2 c5; do
  timeout -k 10 500 python -u bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json
done
timeout -k 10 500 python -u bench.py --config c4 --cpu-sample-docs 32 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
bash profiles/tools/collect.sh c4 --config c4 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c4 gpurun_out/prof_c4/summary.json
