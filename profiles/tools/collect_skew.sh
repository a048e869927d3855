#!/bin/bash
# rocprofv3 evidence for the c3skew line's dominant class (its longest documents, replayed on
# the kHM tier): kernel trace + stats, then separate FETCH_SIZE / WRITE_SIZE passes, each over
# that class alone (bench.py --skew-classes).  Output: gpurun_out/prof_skew_<tag>/.
#   bash profiles/tools/collect_skew.sh <tag> [class]
set -u
tag=$1; cls=${2:-200000}
out=gpurun_out/prof_skew_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --config c3skew --skew-classes $cls --no-cpu --steps 1 --warmup 0 > $out/bench.json 2> $out/bench.err || exit 1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- \
        python3 bench.py --config c3skew --skew-classes $cls --no-cpu --steps 1 --warmup 0 > $out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo done
