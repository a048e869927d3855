#!/bin/sh
# Builds A/B variants of the replay library (same sources, different -D toggles) next to the
# product library; tools/ab_bench.sh times each with bench.py on one GPU box.
set -e
cd "$(dirname "$0")/.."
build() { MT_EXTRA_FLAGS="$2" MT_OUT=fluidframework_amd/libmtreplay_$1.so python fluidframework_amd/build.py --force > /dev/null & }
build base ""
build fullwb "-DMT_FULL_WRITEBACK"
build nolane "-UMT_LANE_ASM"
wait
ls -la fluidframework_amd/libmtreplay_*.so
