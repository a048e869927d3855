"""Diagnostic: the first segment rows that differ from the reference fixture (fast path caps)."""
import sys, os
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import golden_util as gu
import bench
from fluidframework_amd import MergeTreeBatch
name = sys.argv[1] if len(sys.argv) > 1 else "ref_c3_full"
fx = gu.load(name)
interner = gu.interner_for(fx)
a = gu.encode_docs(fx, interner)
caps = bench.capacities(dict(fx["config"]))
mt = MergeTreeBatch(len(fx["docs"]), delta_log_capacity=0, **caps)
mt.load_initial_text(a["seed_off"], a["seed"])
mt.apply_arrays(a)
for i, doc in enumerate(fx["docs"][:2]):
    exp = gu.expected(doc, interner)
    rows, leaves = mt.get_segments(i)
    e = np.asarray(exp["segs"])
    print(name, i, "rows", rows.shape, "exp", e.shape)
    if rows.shape == e.shape:
        bad = np.flatnonzero((rows != e).any(axis=1))
        cols = np.flatnonzero((rows != e).any(axis=0))
        print(" differing rows", len(bad), "cols", cols.tolist())
        for j in bad[:6]:
            print("  ", j, rows[j].tolist(), e[j].tolist())
if os.environ.get("MT_DEBUG_MASK"):
    pass
