"""Register-pressure report of one kernel instantiation (csrc/mt_variants.h name): which
virtual VGPRs stay live through most of the kernel's basic blocks (the values that set the
VGPR budget of a fully inlined op loop), with their defining machine instructions.

    python tools/rp_live.py P_C3 [-DMT_LANE_ASM ...]

Pipeline: hipcc -> device bitcode; llc -stop-after=machine-scheduler -> MIR; llc
-run-pass=amdgpu-print-rp -> per-instruction pressure (pre-RA, virtual registers)."""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLC = "/opt/rocm/lib/llvm/bin/llc"


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    src = os.path.join(REPO, "fluidframework_amd", "_build", "libmtreplay", f"mtk_{name}.hip")
    tmp = f"/tmp/rp_{name}"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-result",
                           "-Wno-unused-value", "--cuda-device-only", "-emit-llvm", "-c", "-o", tmp + ".bc", src] + flags)
    subprocess.check_call([LLC, "-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-O3", "-amdgpu-use-amdgpu-trackers=1",
                           "-stop-after=machine-scheduler", "-o", tmp + ".mir", tmp + ".bc"])
    with open(tmp + ".rp", "w") as fh:
        subprocess.check_call([LLC, "-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-run-pass=amdgpu-print-rp",
                               "-filetype=null", tmp + ".mir"], stdout=fh, stderr=subprocess.STDOUT)
    txt = open(tmp + ".mir").read()
    body = txt[txt.index("\nbody:"):]
    cls = {int(m.group(1)): m.group(2) for m in re.finditer(r"- \{ id: (\d+), class: ([\w_]+)", txt)}
    cnt, masks, bbmax, nb = collections.Counter(), {}, collections.Counter(), 0
    mx = 0
    for line in open(tmp + ".rp"):
        m = re.match(r"\s+(\d+)\s+(\d+)\s", line)
        if m:
            mx = max(mx, int(m.group(2)))
        if line.strip().startswith("Live-thr:"):
            nb += 1
            for m in re.finditer(r"%(\d+):([0-9A-F]+)", line):
                r = int(m.group(1))
                cnt[r] += 1
                masks[r] = masks.get(r, 0) | int(m.group(2), 16)
    thr = int(0.8 * nb)
    rows = [r for r, c in cnt.items() if c >= thr and cls.get(r, "").startswith(("vgpr", "vreg", "av_"))]
    defs = collections.defaultdict(list)
    for line in body.split("\n"):
        m = re.match(r"\s+(?:undef |early-clobber |dead )*%(\d+)(\.[\w]+)?(?::[\w_]+)? = (.*)", line)
        if m and int(m.group(1)) in rows and len(defs[int(m.group(1))]) < 3:
            defs[int(m.group(1))].append((m.group(2) or "") + " " + m.group(3)[:120])
    tot = 0
    for r in sorted(rows, key=lambda r: -cnt[r]):
        n = max(1, bin(masks[r]).count("1") // 2)
        tot += n
        print(r, cls[r], n, cnt[r], " | ".join(defs.get(r, ["?"])))
    print(f"blocks {nb}, max VGPR pressure {mx}, VGPRs live through >= 80% of blocks: {tot}")


if __name__ == "__main__":
    main()
