# A/B of c3skew bench options on one box (product library), each option set in turn:
#   bash tools/ab/ab_skew_args.sh <rounds> "<args 1>" "<args 2>" ...
set -u
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --config c3skew --steps 1 --warmup 1 --no-cpu $a > gpurun_out/absa_$i.json 2> gpurun_out/absa_$i.err || { echo "[$a] failed"; tail -3 gpurun_out/absa_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/absa_$i.json')); print('[$a]', round(d['value']/1e6, 2), d['ms_per_step'], [(c['max_ops'], c['kernel_ms']) for c in d['per_class']], d['parity'])"
  done
done
