# A/B timing of library variants on one box: the C3 12.5k shard, each variant in turn.
#   bash tools/ab/ab.sh <rounds> <variant>...   (variant "head" = libmtreplay.so, else libmtreplay_<v>.so)
set -u
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    lib=fluidframework_amd/libmtreplay_$v.so; [ $v = head ] && lib=fluidframework_amd/libmtreplay.so
    MT_LIB_PATH=$lib timeout -k 10 200 python bench.py --shard 0 --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v failed"; tail -3 gpurun_out/ab_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']/1e6, 2), d['ms_per_step'], d['parity'].get('replay_equals_generation'))"
  done
done
