#!/bin/bash
# Round 3 evidence B: C4 (packed tight tier) bench + rocprofv3 evidence, C5 bench (device
# load + end-to-end leg).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_r3w.json 2> gpurun_out/bench_c4_r3w.err || { tail -n 5 gpurun_out/bench_c4_r3w.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4_r3w.json')); print('c4', d['value'], d['ms_per_step'])"
bash profiles/tools/collect.sh c4 --config c4 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c4 gpurun_out/prof_c4/summary.json > /dev/null || exit 1
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_r3w.json 2> gpurun_out/bench_c5_r3w.err; rc=$?
python -c "import json; d=json.load(open('gpurun_out/bench_c5_r3w.json')); print(d['value'], d['summary_decode']['value'], d['end_to_end'])"
exit $rc
