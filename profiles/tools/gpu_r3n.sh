#!/bin/bash
# Round 3 evidence A: -m gpu suite, smoke, the default bench line (C3, all 100k documents
# on one GPU) and its rocprofv3 evidence (kernel trace + PMC passes).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3v.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_gpu_r3v.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_r3v.json 2> gpurun_out/bench_c3_r3v.err || { tail -20 gpurun_out/bench_c3_r3v.err; exit 1; }
cat gpurun_out/bench_c3_r3v.json
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json > /dev/null || exit 1
echo collected
