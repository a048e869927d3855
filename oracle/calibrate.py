"""CPU-baseline calibration (test infrastructure; build container only, needs /root/reference).

The reference cannot travel to the GPU box, so bench.py times the C restatement
(oracle/mt_oracle.c, `cpu_baseline.kind = "port"`) there.  This script measures, on the same
op streams and one thread each, the reference itself -- the transpiled TypeScript MergeTree
(oracle/_ref, built by oracle/build_ref.py) driven through Client.applyMsg by
oracle/ref_harness.mjs `time` mode under Node -- against the restatement, and writes the ratio
to profiles/<round>/cpu_calibration.json.  The reference is timed twice: with the observer's
position-recording delta callback (what replayDoc records) and with no callback at all (its
fastest replay).  bench.py reports `reference_estimate` = port throughput / the no-callback
ratio, the conservative one (est_reference = restatement / r).

    python oracle/calibrate.py [out.json]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import pyoracle  # noqa: E402
from fluidframework_amd.wire import Batch, Interner, compact_msgs_to_dicts  # noqa: E402

HARNESS = os.path.join(REPO, "oracle", "ref_harness.mjs")
# (config, documents, ops per document): full-length documents of each bench workload, and
# (r6) the long documents of the c3skew classes (the reference pays O(log n) per message
# through its partial lengths, the restatement O(depth) through cached subtree aggregates)
CASES = [("c2", 64, 2000), ("c3", 24, 10000), ("c3", 4, 40000), ("c3", 2, 100000), ("c3", 1, 200000)]


def calibrate(name, ndocs, nops, configs):
    cfg = dict(configs[name], ops=nops)
    with tempfile.TemporaryDirectory() as td:
        cp, gp, tp = (os.path.join(td, f) for f in ("cfg.json", "gen.json", "time.json"))
        json.dump(cfg, open(cp, "w"))
        subprocess.check_call(["node", HARNESS, "gen", cp, "0", str(ndocs), gp])
        subprocess.check_call(["node", HARNESS, "time", gp, tp, "2"])
        ref = json.load(open(tp))
        subprocess.check_call(["node", HARNESS, "time", gp, tp, "2", "nocb"])
        ref_nocb = json.load(open(tp))
        gen = json.load(open(gp))
    b = Batch(Interner(synthetic=True))
    for d in gen["docs"]:
        b.add_doc(d["seed_text"], compact_msgs_to_dicts(d["msgs"]))
    arrays = b.arrays()
    n_ops = int(arrays["doc_off"][-1])
    best = None
    for _ in range(3):
        t = time.perf_counter()
        _, st = pyoracle.replay_batch(arrays, threads=1)
        t = time.perf_counter() - t
        best = t if best is None else min(best, t)
    assert (st == 0).all()
    port = n_ops / best
    return dict(docs=ndocs, ops_per_doc=nops, ops=n_ops, threads=1,
                reference_ops_per_s=round(ref["ops_per_s"], 1),
                reference_nocb_ops_per_s=round(ref_nocb["ops_per_s"], 1),
                reference_runtime=f"node {ref['node']}",
                port_ops_per_s=round(port, 1), ratio_port_over_reference=round(port / ref["ops_per_s"], 3),
                ratio_port_over_reference_nocb=round(port / ref_nocb["ops_per_s"], 3))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r6", "cpu_calibration.json")
    configs = json.load(open(os.path.join(REPO, "bench", "configs.json")))
    res = {"note": "one thread each, same op streams: the transpiled reference MergeTree (Client.applyMsg, "
                   "observer with the position-recording delta callback / with no callback) under Node vs "
                   "oracle/mt_oracle.c as bench.py times it; measured in the build container by "
                   "oracle/calibrate.py"}
    for name, nd, no in CASES:
        key = name if no <= 10000 else f"{name}_{no // 1000}k"
        res[key] = calibrate(name, nd, no, configs)
        print(key, res[key], flush=True)
        json.dump(res, open(out, "w"), indent=1)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
