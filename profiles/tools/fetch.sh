# FETCH_SIZE calibration on the replay kernel's read patterns (profiles/tools/fetch_probe.hip):
#   bash profiles/tools/fetch.sh   (GPU box; writes gpurun_out/fp/calibration.json)
set -u
mkdir -p gpurun_out/fp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 profiles/tools/fetch_probe > gpurun_out/fp/expected.jsonl || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fp/p1 -o run -- profiles/tools/fetch_probe > gpurun_out/fp/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/fp/p2 -o run -- profiles/tools/fetch_probe > gpurun_out/fp/p2.log 2>&1 || exit 1
python3 profiles/tools/fetch_probe.py gpurun_out/fp > gpurun_out/fp/calibration.json
