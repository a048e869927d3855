#!/bin/bash
# occupancy probe at the default C3 shard: paged LDS footprint (documents per CU) x VGPR budget
set -u
mkdir -p gpurun_out
run() {  # tag caps
  timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --page-caps $2 > gpurun_out/occ_$1.json 2>gpurun_out/occ_$1.err || { echo "$1 failed"; tail -2 gpurun_out/occ_$1.err; return 0; }
  python -c "import json; d=json.load(open('gpurun_out/occ_$1.json')); print('$1 $2', d['value'], d['roofline']['kernel_ms'], d['parity']['replay_equals_generation'])"
}
run w3_10cu 208,240,224
run w3_9cu 224,288,288
run w3_8cu 256,320,320
MT_EXTRA_FLAGS="-DMT_PAGED_WAVES=0" timeout -k 10 300 python fluidframework_amd/build.py --force > gpurun_out/occ_build.log 2>&1 || { tail -3 gpurun_out/occ_build.log; exit 1; }
run w0_10cu 208,240,224
run w0_8cu 256,320,320
