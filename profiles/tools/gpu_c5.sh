set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "snapshot" > gpurun_out/pytest_snap2.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_snap2.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config c5 --docs 20000 --steps 3 > gpurun_out/c5_20k.json 2>gpurun_out/c5_20k.err || { tail -20 gpurun_out/c5_20k.err; exit 1; }
cat gpurun_out/c5_20k.json
timeout -k 10 500 python -u bench.py --config c5 --steps 3 > gpurun_out/c5_full.json 2>gpurun_out/c5_full.err || { tail -20 gpurun_out/c5_full.err; exit 1; }
cat gpurun_out/c5_full.json
