set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "snapshot" > gpurun_out/pytest_snap.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_snap.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu3.log
timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > gpurun_out/bench_h96.json 2>gpurun_out/bench_h96.err && cat gpurun_out/bench_h96.json
