set -u
mkdir -p gpurun_out
MT_EXTRA_FLAGS="-DMT_PROF" timeout -k 10 300 python fluidframework_amd/build.py --force > gpurun_out/prof_build.log 2>&1 || { tail gpurun_out/prof_build.log; exit 1; }
timeout -k 10 300 python -u tests/debug_prof.py c3 10000 2048 > gpurun_out/prof_c3.txt 2>&1 || { tail -20 gpurun_out/prof_c3.txt; exit 1; }
cat gpurun_out/prof_c3.txt
