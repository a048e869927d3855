set -u
mkdir -p gpurun_out
for n in 2048 4096 4864 5120 8192 10000 20000; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 3 --docs $n > gpurun_out/ds_$n.json 2>gpurun_out/ds_$n.err || { echo "bench $n failed"; tail gpurun_out/ds_$n.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ds_$n.json')); print('docs $n', d['value'], d['roofline']['kernel_ms'])"
done
