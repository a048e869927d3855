#!/bin/sh
# A/B of the sliced paged schedule (mt_options.paged_slices) on the C3 shard, then its parity test.
run() { # name lib slices
  MT_LIB_PATH=fluidframework_amd/libmtreplay_$2.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --paged-slices $3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -5 gpurun_out/ab_$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', d['value'], d['ms_per_step'], d['parity'], d['roofline']['docs_replayed_from_hbm']['total'])"
}
MT_LIB_PATH=fluidframework_amd/libmtreplay_slice.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "sliced or tight_tier or full_streams" > gpurun_out/pytest_slice.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_slice.log
[ $rc -eq 0 ] || exit $rc
run head head 0 && run s0 slice 0 && run s16 slice 16 && run s8 slice 8 && run head2 head 0 && run s16b slice 16 && run s32 slice 32
