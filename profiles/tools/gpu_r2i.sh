#!/bin/bash
# Round-2 HEAD check after the PagedSlice kernel entry: -m gpu suite, smoke, C3 rocprofv3
# evidence (trace + PMC passes), default bench line with CPU leg, live and C5 lines.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_i.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_i.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_i.json 2> gpurun_out/bench_c3_i.err || { tail -20 gpurun_out/bench_c3_i.err; exit 1; }
cat gpurun_out/bench_c3_i.json
timeout -k 10 500 python -u bench.py --config live --steps 3 --warmup 1 > gpurun_out/bench_live_i.json 2> gpurun_out/bench_live_i.err || { tail -20 gpurun_out/bench_live_i.err; exit 1; }
cat gpurun_out/bench_live_i.json
timeout -k 10 600 python -u bench.py --config c5 > gpurun_out/bench_c5_i.json 2> gpurun_out/bench_c5_i.err || { tail -20 gpurun_out/bench_c5_i.err; exit 1; }
cat gpurun_out/bench_c5_i.json
