#!/bin/bash
# the other configurations on the current build (perf-log rows)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > gpurun_out/o_c2.json 2>gpurun_out/o_c2.err || { tail -5 gpurun_out/o_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c4 --docs 1024 --no-cpu --steps 2 > gpurun_out/o_c4.json 2>gpurun_out/o_c4.err || { tail -5 gpurun_out/o_c4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 --no-cpu --steps 3 > gpurun_out/o_c5.json 2>gpurun_out/o_c5.err || { tail -5 gpurun_out/o_c5.err; exit 1; }
for f in c2 c4 c5; do python -c "import json; d=json.load(open('gpurun_out/o_$f.json')); print('$f', d['value'], d['unit'], d['ms_per_step'], d.get('parity'))"; done
