# A/B of library variants on one bench config (no CPU leg, no ingest), each variant in turn:
#   bash tools/ab/ab_cfg.sh <config> <rounds> <variant>...   (variant "head" = libmtreplay.so)
set -u
mkdir -p gpurun_out
cfg=$1; rounds=$2; shift 2
for r in $(seq $rounds); do
  for v in "$@"; do
    lib=fluidframework_amd/libmtreplay_$v.so; [ $v = head ] && lib=fluidframework_amd/libmtreplay.so
    MT_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu --no-ingest > gpurun_out/abc_$v.json 2> gpurun_out/abc_$v.err || { echo "$v failed"; tail -3 gpurun_out/abc_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abc_$v.json')); print('$v', round(d['value']/1e6, 3), d['ms_per_step'], d['parity'])"
  done
done
