set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu2.log
for cap in 192 160 128 112 96; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 5 --lds-cap $cap > gpurun_out/sweep_$cap.json 2>gpurun_out/sweep_$cap.err || { echo "bench $cap failed"; tail gpurun_out/sweep_$cap.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_$cap.json')); print($cap, d['value'], d['roofline']['kernel_ms'], d['roofline']['docs_replayed_from_hbm'], d['parity']['replay_equals_generation'])"
done
