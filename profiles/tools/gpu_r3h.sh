#!/bin/bash
# Round 3: growth step (documents beyond the handle's paged capacities move to larger HBM
# regions) + summary paths (sliced catch-up) + the C5 bench with its end-to-end leg.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "growth or grow" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3h_grow.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/pytest_r3h_grow.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_snapdec.py -m gpu -x -q -k "snapshot or summaries or catch_up" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3h_snap.log 2>&1; rc=$?
tail -n 5 gpurun_out/pytest_r3h_snap.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_r3h.json 2> gpurun_out/bench_c5_r3h.err; rc=$?
tail -n 3 gpurun_out/bench_c5_r3h.err
python -c "import json; d=json.load(open('gpurun_out/bench_c5_r3h.json')); print(d['value'], d['summary_decode']['value'], d['end_to_end'])"
exit $rc
