#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- build the reference merge-tree into oracle/_ref/.

Transpiles (with oracle/ts2js.py) the reference's own TypeScript sources where they lie
under /root/reference/packages/dds/merge-tree/src (and its test helpers) into ES modules
under oracle/_ref/.  Output is git-ignored and listed in .gpurunignore: the reference
never travels to the GPU box.  Nothing is copied into the repository.

Usage:  python3 oracle/build_ref.py [--ref /root/reference]
"""
import argparse
import glob
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from ts2js import transpile_tree  # noqa: E402

SHIMS = {
    "@fluidframework/common-utils": "common-utils.mjs",
    "@fluidframework/protocol-definitions": "protocol-definitions.mjs",
    "@fluidframework/telemetry-utils": "telemetry-utils.mjs",
    "@fluidframework/container-definitions": "container-definitions.mjs",
    "@fluidframework/test-runtime-utils": "test-runtime-utils.mjs",
}
TYPE_ONLY = {"@fluidframework/core-interfaces", "@fluidframework/datastore-definitions",
             "@fluidframework/common-definitions", "@fluidframework/runtime-utils"}
NODE_BUILTINS = {"assert", "fs", "path", "perf_hooks"}

# test helpers and the known-answer / farm specs that pin the hot path (random-js, a
# test-only npm dependency absent here, is replaced by oracle/shims/random-js.mjs).
TEST_FILES = [
    "index.ts", "mergeTreeOperationRunner.ts", "client.conflictFarm.spec.ts",
    "client.reconnectFarm.spec.ts", "testClient.ts", "testClientLogger.ts", "testServer.ts", "testUtils.ts",
    "mergeTree.markRangeRemoved.spec.ts", "mergeTree.annotate.spec.ts",
    "mergeTree.insertingWalk.spec.ts", "mergeTree.insert.deltaCallback.spec.ts",
    "mergeTree.markRangeRemoved.deltaCallback.spec.ts", "mergeTree.annotate.deltaCallback.spec.ts",
    "client.applyMsg.spec.ts", "properties.spec.ts", "snapshot.spec.ts", "snapshotlegacy.spec.ts",
    "client.spec.ts", "client.walkSegments.spec.ts", "segmentGroupCollection.spec.ts",
    "collections.list.spec.ts", "tracking.spec.ts", "resetPendingSegmentsToOp.spec.ts",
    "client.localReference.spec.ts",
]


SEQ_FILES = ["sequenceDeltaEvent.ts"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "_ref"))
    args = ap.parse_args()
    src_dir = os.path.join(args.ref, "packages/dds/merge-tree/src")
    if not os.path.isdir(src_dir):
        print(f"reference not found at {src_dir}; skipping", file=sys.stderr)
        return 1
    files = {}
    for p in sorted(glob.glob(os.path.join(src_dir, "*.ts"))):
        mod = "mt/" + os.path.basename(p)[:-3]
        files[mod] = (p, open(p, encoding="utf-8").read())
    for name in TEST_FILES:
        p = os.path.join(src_dir, "test", name)
        if os.path.exists(p):
            files["mt/test/" + name[:-3]] = (p, open(p, encoding="utf-8").read())
    # the sequence package's event objects (SequenceDeltaEvent / SequenceMaintenanceEvent:
    # ranges sorted and deduplicated by segment ordinal through SortedSegmentSet) -- the
    # reference side of the GPU facade's event parity (oracle/ref_harness.mjs events)
    seq_dir = os.path.join(args.ref, "packages/dds/sequence/src")
    for name in SEQ_FILES:
        p = os.path.join(seq_dir, name)
        files["seq/" + name[:-3]] = (p, open(p, encoding="utf-8").read())

    def resolve(from_mod, spec):
        if spec == "@fluidframework/merge-tree":
            return "mt/index"
        if spec in SHIMS:
            return ("shim", os.path.relpath(os.path.join("shims", SHIMS[spec]),
                                            os.path.dirname(from_mod)))
        if spec in TYPE_ONLY:
            return ("shim", os.path.relpath("shims/empty.mjs", os.path.dirname(from_mod)))
        if spec in NODE_BUILTINS:
            return ("shim", spec)
        if spec == "random-js":
            return ("shim", os.path.relpath("shims/random-js.mjs", os.path.dirname(from_mod)))
        if spec.startswith("."):
            base = os.path.normpath(os.path.join(os.path.dirname(from_mod), spec))
            if base in files:
                return base
            if base + "/index" in files:
                return base + "/index"
            if spec in ("./", "."):
                return os.path.normpath(os.path.join(os.path.dirname(from_mod), "index"))
            raise KeyError(f"{from_mod}: cannot resolve {spec}")
        raise KeyError(f"{from_mod}: unknown module {spec}")

    out = transpile_tree(files, resolve)
    if os.path.isdir(args.out):
        shutil.rmtree(args.out)
    os.makedirs(os.path.join(args.out, "shims"))
    for f in glob.glob(os.path.join(HERE, "shims", "*.mjs")):
        shutil.copy(f, os.path.join(args.out, "shims"))
    with open(os.path.join(args.out, "shims", "empty.mjs"), "w") as fh:
        fh.write("export {};\n")
    for mod, js in out.items():
        path = os.path.join(args.out, mod + ".mjs")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w", encoding="utf-8") as fh:
            fh.write(js)
    with open(os.path.join(args.out, "package.json"), "w") as fh:
        fh.write('{"type": "module"}\n')
    print(f"transpiled {len(out)} modules into {args.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
