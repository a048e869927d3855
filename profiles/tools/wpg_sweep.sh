set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu6.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu6.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu6.log | head -20; exit 1; }
for w in 1 2; do
  MT_WPG=$w timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > gpurun_out/wpg_$w.json 2>gpurun_out/wpg_$w.err || { echo "bench $w failed"; tail gpurun_out/wpg_$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/wpg_$w.json')); print('wpg $w', d['value'], d['roofline']['kernel_ms'], d['roofline']['docs_replayed_from_hbm']['total'], d['parity']['replay_equals_generation'])"
done
for n in 4096 4608 5120; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 3 --docs $n > gpurun_out/ds2_$n.json 2>/dev/null && python -c "import json,sys; d=json.load(open('gpurun_out/ds2_$n.json')); print('docs $n', d['value'], d['roofline']['kernel_ms'])"
done
