"""Scale check on the GPU: generate N C3 documents, replay them, compare the replay's
checksums with the generation's; for mismatching documents re-run each alone (docs=1 at the
same global index) to tell a scale effect from a per-document one.
    python tools/check_scale.py N [n_isolated]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402


def run(cfg, docs, base):
    caps = bench.capacities(cfg)
    mt = MergeTreeBatch(docs, **caps)
    batch = mt.generate(cfg, base)
    gst = mt.status().copy()
    gen = mt.checksums().copy()
    gpk = mt.last_paged_peaks()
    seed_off, seed = mt.generated_seeds(cfg, base)
    mt.load_initial_text(seed_off, seed)
    mt.reset()
    batch.apply_async()
    mt.sync()
    rst = mt.status().copy()
    rep = mt.checksums().copy()
    return gen, gst, rep, rst, gpk, mt.last_paged_peaks()


def main():
    n = int(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cfg = dict(json.load(open(os.path.join(REPO, "bench", "configs.json")))["c3"])
    gen, gst, rep, rst, gpk, rpk = run(cfg, n, 0)
    bad = np.nonzero((gen != rep) | (gst != 0) | (rst != 0))[0]
    print("docs", n, "gen peaks", gpk, "replay peaks", rpk, flush=True)
    print("gen status", np.unique(gst, return_counts=True), "replay status", np.unique(rst, return_counts=True))
    print("mismatching docs", len(bad), bad[:40].tolist(), flush=True)
    for f in gen.dtype.names:
        print(" field", f, "differs in", int((gen[f] != rep[f]).sum()))
    for d in bad[:k].tolist():
        g1, gs1, r1, rs1, _, _ = run(cfg, 1, d)
        print(f"doc {d}: alone gen==big gen {bool(g1[0] == gen[d])} alone rep==alone gen {bool(r1[0] == g1[0])} "
              f"big rep==alone gen {bool(rep[d] == g1[0])} status {gs1[0]},{rs1[0]} big {gst[d]},{rst[d]}", flush=True)


if __name__ == "__main__":
    main()
