set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c3 --docs 2048 --no-cpu --steps 2 --warmup 1 > gpurun_out/c3_2048.json 2>gpurun_out/c3_2048.err || { tail -20 gpurun_out/c3_2048.err; exit 1; }
cat gpurun_out/c3_2048.json
timeout -k 10 400 python -u bench.py --config c4 --docs 1024 --no-cpu --steps 2 --warmup 1 > gpurun_out/c4_1024.json 2>gpurun_out/c4_1024.err || { tail -20 gpurun_out/c4_1024.err; exit 1; }
cat gpurun_out/c4_1024.json
