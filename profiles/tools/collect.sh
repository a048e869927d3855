#!/bin/bash
# Collects the rocprofv3 evidence for one bench configuration on the GPU box.
#   bash profiles/tools/collect.sh <tag> [bench args other than --steps/--warmup...]
# (--no-ingest: the ingest pipeline's own small replays would mix into the per-step figures)
# 1) kernel trace + stats of the bench run (CSV), 2) separate --pmc passes (SQ instruction
# mix, SQ stall split, LDS bank conflicts, HBM FETCH_SIZE, HBM WRITE_SIZE, and the L2's
# memory-side request counts that FETCH_SIZE derives from, for the correction check).  Output goes to
# gpurun_out/prof_<tag>/; profiles/tools/summarize.py turns it into a JSON summary.
set -u
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --no-cpu --no-ingest --steps 5 --warmup 1 "$@" > $out/bench.json 2> $out/bench.err || exit 1
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- \
        python3 bench.py --no-cpu --no-ingest --steps 1 --warmup 0 "$@" > $out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo done
