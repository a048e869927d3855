# One GPU call of this round's checks: the -m gpu suite, then optional A/B rounds of library
# variants on the C3 shard (tools/ab/ab.sh), each step under its own time limit; stops at the
# first failure.  Logs under gpurun_out/.
#   bash tools/gpu_step.sh <tag> [tests|notests] [ab_rounds variant...]
set -u
tag=$1; shift
mkdir -p gpurun_out
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 1300 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -rs \
    > gpurun_out/${tag}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
  tail -3 gpurun_out/${tag}_pytest.log
fi
shift || true
if [ $# -gt 1 ]; then
  bash tools/ab/ab.sh "$@" > gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 1; }
  cat gpurun_out/${tag}_ab.log
fi
# optional: GPU_SKEW=1 runs the c3skew line after the A/B (one step)
if [ "${GPU_SKEW:-0}" = 1 ]; then
  timeout -k 10 900 python -u bench.py --config c3skew --steps 1 --warmup 0 > gpurun_out/${tag}_skew.json 2> gpurun_out/${tag}_skew.err \
    || { echo "c3skew failed"; tail -5 gpurun_out/${tag}_skew.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${tag}_skew.json')); print('c3skew', round(d['value']/1e6,2), d['ms_per_step'], d['parity'], [(c['max_ops'], c['kernel_ms']) for c in d['per_class']])"
fi
