#!/bin/bash
# One GPU-box session: the -m gpu parity suite, the default bench line, then (optional
# tag) the rocprofv3 evidence of profiles/tools/collect.sh.  Every GPU step has its own
# time limit and the chain stops at the first failure.
#   bash profiles/tools/gpu_check.sh [tag [bench args...]]
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || {
    echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ $# -ge 1 ]; then
    tag=$1; shift
    bash profiles/tools/collect.sh "$tag" "$@" || exit 1
fi
echo all-done
