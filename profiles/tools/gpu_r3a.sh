#!/bin/bash
# Round-3 first check: -m gpu suite (incl. the new sliced-without-LDS-tier and RCCL world-1
# tests), smoke, the default bench line (now the metric's whole 100k-document C3 job on one
# GPU) and its rocprofv3 evidence (kernel trace + PMC passes at the same configuration).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3a.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_r3a.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_r3a.json 2> gpurun_out/bench_c3_r3a.err || { tail -20 gpurun_out/bench_c3_r3a.err; exit 1; }
cat gpurun_out/bench_c3_r3a.json
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json || exit 1
