"""Builds the HIP replay library in-tree (fluidframework_amd/libmtreplay.so) for gfx950, and the
host summary decoder (libmtsnapdec.so).
hipcc cross-compiles here without a GPU; the .so travels to the GPU box with the repo."""
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "mt_replay.hip")
VARIANTS_H = os.path.join(HERE, "csrc", "mt_variants.h")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("mt_replay.hip", "mt_engine.h", "mt_device.h", "mt_paged.h",
                                                 "mt_kernels.h", "mt_variants.h")] + [
    os.path.join(os.path.dirname(HERE), "include", f) for f in ("mt_replay.h", "mt_types.h")]
OBJ_DIR = os.path.join(HERE, "_build")
OUT = os.environ.get("MT_OUT") or os.path.join(HERE, "libmtreplay.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -amdgpu-use-amdgpu-trackers: the scheduler's AMDGPU register-pressure trackers (A/B on the
# C3 bench, same registers and spills: 886 -> 870 ms per step; profiles/r2/ab_flags.log)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wno-unused-result",
         "-Wno-unused-value", "-mllvm", "-amdgpu-use-amdgpu-trackers=1"] + os.environ.get("MT_EXTRA_FLAGS", "").split()


# Per-instantiation compile options (the generated translation unit's first lines, e.g.
# {"P_C3": "#define MT_PAGED_WAVES 4\n"}); none in the product build -- round 6 A/B'd the C3 tier
# at 4 waves per SIMD and found it slower (profiles/README.md).  MT_NO_VARIANT_DEFINES=1 drops
# them; MT_SINGLE_TU=1 builds ignore them.
VARIANT_DEFINES = {}

# what the kernel instantiations (mtk_*.o) compile from: not mt_replay.hip's host code
KERNEL_DEPS = [p for p in DEPS if not p.endswith("mt_replay.hip")]


def _fresh(obj, deps):
    """obj exists and is newer than every dependency (and than this build script's flags)."""
    if not os.path.exists(obj):
        return False
    t = os.path.getmtime(obj)
    return all(os.path.getmtime(d) <= t for d in deps + [os.path.abspath(__file__)])


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in DEPS)


def variants():
    """(name, kernel expression) of every kernel instantiation in csrc/mt_variants.h."""
    text = open(VARIANTS_H).read()
    return re.findall(r"X\((\w+), \((.*?)\)\)\s*\\?\n", text)


def build(force=False, verbose=False):
    """One translation unit per kernel instantiation (csrc/mt_variants.h) plus the host side,
    compiled in parallel and linked into one shared library (MT_SINGLE_TU=1: the whole library
    as one translation unit)."""
    if not force and not needs_build():
        return OUT
    single = os.environ.get("MT_SINGLE_TU") == "1"
    if single:
        cmd = [HIPCC] + FLAGS + ["-DMT_SINGLE_TU", "-o", OUT + ".tmp", SRC]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        os.replace(OUT + ".tmp", OUT)
        return OUT
    tag = os.path.splitext(os.path.basename(OUT))[0]   # variant libraries (MT_OUT) build apart
    obj_dir = os.path.join(OBJ_DIR, tag)
    os.makedirs(obj_dir, exist_ok=True)
    # objects built with other flags are rebuilt; the stamp names the flags only once a build
    # with them has linked (an interrupted rebuild must not leave old-flag objects looking fresh)
    stamp = os.path.join(obj_dir, "flags.txt")
    if not os.path.exists(stamp) or open(stamp).read() != " ".join(FLAGS):
        force = True
        if os.path.exists(stamp):
            os.remove(stamp)
    # MT_ONLY=P_C3,P_C4: an A/B variant that recompiles only those kernels; the other objects
    # come from the product build (_build/libmtreplay)
    only = [x for x in os.environ.get("MT_ONLY", "").split(",") if x]
    cflags = [f for f in FLAGS if f != "-shared"] + ["-c"]
    jobs = [(SRC, os.path.join(obj_dir, "mt_replay.o"))]
    link_only = []
    if not force and not os.environ.get("MT_ONLY") and _fresh(jobs[0][1], DEPS):
        link_only.append(jobs.pop()[1])
    for name, expr in variants():
        src = os.path.join(obj_dir, f"mtk_{name}.hip")
        body = (("" if os.environ.get("MT_NO_VARIANT_DEFINES") else VARIANT_DEFINES.get(name, "")) +
                f'#include "{os.path.join(HERE, "csrc", "mt_kernels.h")}"\n'
                f'#include "{os.path.join(HERE, "csrc", "mt_variants.h")}"\n'
                f"const void *mtk_{name}() {{ return (const void *)({expr}); }}\n")
        if not os.path.exists(src) or open(src).read() != body:
            with open(src, "w") as fh:
                fh.write(body)
        obj = os.path.join(obj_dir, f"mtk_{name}.o")
        if not force and not only and _fresh(obj, [src] + KERNEL_DEPS):   # (mt_replay.hip is host code)
            link_only.append(obj)
            continue
        if only and name not in only:
            base_obj = os.path.join(OBJ_DIR, "libmtreplay", f"mtk_{name}.o")
            if os.path.abspath(base_obj) != os.path.abspath(obj):
                shutil.copyfile(base_obj, obj)
            link_only.append(obj)
            continue
        jobs.append((src, obj))
    par = int(os.environ.get("MT_BUILD_JOBS") or min(8, os.cpu_count() or 1))
    running, done = [], []
    pending = list(jobs)
    while pending or running:
        while pending and len(running) < par:
            src, obj = pending.pop(0)
            cmd = [HIPCC] + cflags + ["-o", obj, src]
            if verbose:
                print(" ".join(cmd))
            running.append((subprocess.Popen(cmd), src))
        p, src = running.pop(0)
        if p.wait() != 0:
            for q, _ in running:
                q.wait()
            raise subprocess.CalledProcessError(p.returncode, src)
        done.append(src)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + [o for _, o in jobs] + link_only
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    with open(stamp, "w") as fh:
        fh.write(" ".join(FLAGS))
    return OUT


SNAP_SRC = os.path.join(HERE, "csrc", "mt_snapdec.cpp")
SNAP_OUT = os.path.join(HERE, "libmtsnapdec.so")


def build_snapdec(force=False, verbose=False):
    """The host summary decoder (include/mt_snapshot.h), plain g++ (no device code)."""
    deps = [SNAP_SRC] + [os.path.join(os.path.dirname(HERE), "include", f) for f in ("mt_snapshot.h", "mt_types.h")]
    if not force and os.path.exists(SNAP_OUT) and all(os.path.getmtime(d) <= os.path.getmtime(SNAP_OUT) for d in deps):
        return SNAP_OUT
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-o", SNAP_OUT + ".tmp", SNAP_SRC, "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(SNAP_OUT + ".tmp", SNAP_OUT)
    return SNAP_OUT


def build_node_addon(verbose=False):
    """The N-API addon for the Node facade (fluidframework_amd/js); skipped without Node headers."""
    js = os.path.join(HERE, "js")
    out = os.path.join(js, "mtreplay.node")
    if not os.path.exists("/usr/include/node/node_api.h"):
        return None
    build_snapdec(verbose=verbose)
    deps = [os.path.join(js, "binding.cc"), OUT, SNAP_OUT]
    if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    if verbose:
        print("sh", os.path.join(js, "build.sh"))
    subprocess.check_call(["sh", os.path.join(js, "build.sh")])
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    if not os.environ.get("MT_OUT"):   # variant libraries (MT_OUT) leave the addon alone
        build_node_addon(verbose=True)
        build_snapdec(verbose=True)
    print(OUT)
