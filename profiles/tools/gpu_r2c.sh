#!/bin/bash
# Live-client tests (incl. markers), then the rocprofv3 evidence for the default C3 workload.
set -u
mkdir -p gpurun_out
bash profiles/tools/gpu_live.sh || exit 1
bash profiles/tools/collect.sh c3 || exit 1
python profiles/tools/summarize.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary.json
