#!/bin/bash
# Round 3: C3 shard A/B -- round-start library, head (growth step, bool pg_room in the loop),
# head without the big-region lookup (-DMT_AB_NOBIG) -- and the C5 end-to-end debug probe.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_c5e2e.py > gpurun_out/debug_c5e2e.txt 2>&1; echo "c5 debug rc=$?"; tail -n 20 gpurun_out/debug_c5e2e.txt
for i in 1 2; do
  for v in base head nobig; do
    lib=$PWD/fluidframework_amd/libmtreplay.so
    [ $v = base ] && lib=$PWD/bench_libs/libmt_base.so
    [ $v = nobig ] && lib=$PWD/bench_libs/libmt_nobig.so
    MT_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --shard 0 --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_r3k_${v}_$i.json 2> gpurun_out/ab_r3k_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_r3k_${v}_$i.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
