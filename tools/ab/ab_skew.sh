# A/B timing of library variants on the c3skew line (no CPU leg), each variant in turn.
#   bash tools/ab/ab_skew.sh <rounds> <variant>...   (variant "head" = libmtreplay.so, else libmtreplay_<v>.so)
set -u
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    lib=fluidframework_amd/libmtreplay_$v.so; [ $v = head ] && lib=fluidframework_amd/libmtreplay.so
    MT_LIB_PATH=$lib timeout -k 10 300 python bench.py --config c3skew --steps 1 --warmup 1 --no-cpu > gpurun_out/abs_$v.json 2> gpurun_out/abs_$v.err || { echo "$v failed"; tail -3 gpurun_out/abs_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abs_$v.json')); print('$v', round(d['value']/1e6, 2), d['ms_per_step'], [(c['max_ops'], c['kernel_ms']) for c in d['per_class']], d['parity'])"
  done
done
