# Register / spill report of kernel instantiations (csrc/mt_variants.h names), device code only:
#   bash tools/regs.sh P_C3 P_FULL
set -eu
cd "$(dirname "$0")/.."
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -Wno-unused-value \
    -mllvm -amdgpu-use-amdgpu-trackers=1 --cuda-device-only -c -o /tmp/regs_$v.o \
    -Rpass-analysis=kernel-resource-usage fluidframework_amd/_build/libmtreplay/mtk_$v.hip 2>&1 |
    grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size" | sed "s/^.*remark: //" | sed "s/^/$v /"
done
