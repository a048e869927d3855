#!/bin/bash
# Round 3: summary-load paths after the decoder rework (parallel fetch, range uploads):
# the snapshot / summary tests incl. the sliced catch-up, then the C5 bench with its
# end-to-end leg (JSON bytes -> replayed tails).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_snapdec.py -m gpu -x -q -k "snapshot or summaries or catch_up" --timeout 300 --timeout-method thread > gpurun_out/pytest_r3g.log 2>&1; rc=$?
tail -n 5 gpurun_out/pytest_r3g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_r3g.json 2> gpurun_out/bench_c5_r3g.err; rc=$?
tail -n 3 gpurun_out/bench_c5_r3g.err
python -c "import json; d=json.load(open('gpurun_out/bench_c5_r3g.json')); print(d['value'], d['summary_decode']['value'], d['end_to_end'])"
exit $rc
