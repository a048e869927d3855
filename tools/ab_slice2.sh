#!/bin/sh
run() { # name lib slices
  MT_LIB_PATH=fluidframework_amd/libmtreplay_$2.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --paged-slices $3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -5 gpurun_out/ab_$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', d['value'], d['ms_per_step'])"
}
run s0a slice 0 && run heada head 0 && run s0b slice 0 && run headb head 0 && run s4 slice 4
