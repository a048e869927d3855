#!/bin/bash
# C4 (64 writers, lag 1000) at its full 4096 documents: tight vs loose paged capacities
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config c4 --no-cpu --steps 2 > gpurun_out/c4_tight.json 2>gpurun_out/c4_tight.err || { tail -5 gpurun_out/c4_tight.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4_tight.json')); print('tight', d['value'], d['ms_per_step'], d['roofline']['paged_peaks'], d['roofline']['paged_caps'], d['parity'])"
timeout -k 10 500 python -u bench.py --config c4 --no-cpu --steps 2 --page-caps 393,2560,2560 > gpurun_out/c4_loose.json 2>gpurun_out/c4_loose.err || { tail -5 gpurun_out/c4_loose.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4_loose.json')); print('loose', d['value'], d['ms_per_step'], d['parity'])"
