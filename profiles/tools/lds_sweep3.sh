set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu5.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu5.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu5.log | head -20; exit 1; }
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --steps 5 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || { echo "bench $tag failed"; tail gpurun_out/sw_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_$tag.json')); print('$tag', d['value'], d['roofline']['kernel_ms'], d['roofline']['docs_replayed_from_hbm']['total'], d['parity']['replay_equals_generation'])"
}
run c192 --lds-cap 192
run c184 --lds-cap 184
run c176 --lds-cap 176
