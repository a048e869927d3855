#!/bin/sh
# Builds A/B variants of the replay library (same sources, different compiler flags or -D
# toggles) next to the product library; tools/ab_bench.sh times each with bench.py on one
# GPU box.   sh tools/build_variants.sh name1 "flags1" name2 "flags2" ...
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  MT_EXTRA_FLAGS="$2" MT_OUT=fluidframework_amd/libmtreplay_$1.so python fluidframework_amd/build.py --force > /dev/null &
  shift 2
done
wait
ls -la fluidframework_amd/libmtreplay_*.so
