set -u
mkdir -p gpurun_out
MT_EXTRA_FLAGS="-DMT_PROF -DMT_PROF2" timeout -k 10 300 python fluidframework_amd/build.py --force > gpurun_out/prof_build.log 2>&1 || { tail gpurun_out/prof_build.log; exit 1; }
timeout -k 10 300 python -u tests/debug_prof.py c2 2000 10000 > gpurun_out/prof2_c2.txt 2>&1 || { tail -20 gpurun_out/prof2_c2.txt; exit 1; }
cat gpurun_out/prof2_c2.txt
