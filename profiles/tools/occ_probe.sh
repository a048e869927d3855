#!/bin/bash
# occupancy probe: documents per CU (paged LDS footprint) x VGPR budget, C3 mix at 5000 ops
set -u
mkdir -p gpurun_out
run() {  # tag caps
  timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --ops 5000 --page-caps $2 > gpurun_out/occ_$1.json 2>gpurun_out/occ_$1.err || { echo "$1 failed"; tail -2 gpurun_out/occ_$1.err; return 0; }
  python -c "import json; d=json.load(open('gpurun_out/occ_$1.json')); print('$1 $2', d['value'], d['roofline']['kernel_ms'], d['roofline']['paged_peaks'], d['parity']['replay_equals_generation'])"
}
run base_A 208,240,224
MT_EXTRA_FLAGS="-DMT_PAGED_WAVES=3" timeout -k 10 300 python fluidframework_amd/build.py --force > gpurun_out/occ_build.log 2>&1 || { tail -3 gpurun_out/occ_build.log; exit 1; }
run w3_A 208,240,224
run w3_B 120,240,224
run w3_C 112,224,192
