"""Golden maintenance-event counts, made by the reference itself.

For every replay fixture (tests/golden/ref_*.json.gz made by make_golden.py) the transpiled
reference (oracle/build_ref.py -> oracle/_ref) replays each document's message stream through
Client.applyMsg with a mergeTreeMaintenanceCallback attached (oracle/ref_harness.mjs "maint"
mode) and records per document [SPLIT, APPEND, UNLINK] counts
(MT/mergeTreeDeltaCallback.ts:15-35).  Output: tests/golden/ref_maint.json (data only)."""
import gzip
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
FIXTURES = ["ref_small", "ref_c2", "ref_c3", "ref_c4", "ref_ext", "ref_ext_long", "ref_farm", "ref_c3_full",
            "ref_c4_full"]


def main():
    if not os.path.isdir(os.path.join(REPO, "oracle", "_ref")):
        subprocess.check_call([sys.executable, os.path.join(REPO, "oracle", "build_ref.py")])
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name in FIXTURES:
            with gzip.open(os.path.join(HERE, name + ".json.gz"), "rt") as f:
                fx = json.load(f)
            ip, op = os.path.join(td, "in.json"), os.path.join(td, "out.json")
            with open(ip, "w") as f:
                json.dump({"docs": fx["docs"]}, f)
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "maint", ip, op])
            with open(op) as f:
                out[name] = json.load(f)
    with open(os.path.join(HERE, "ref_maint.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
