"""Diagnostic: rows of ref_c3_full doc 0 at the bench capacities, with and without a props
capacity that forces the hand-over to the growth step."""
import sys, os
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import golden_util as gu
import bench
from fluidframework_amd import MergeTreeBatch
fx = gu.load("ref_c3_full")
interner = gu.interner_for(fx)
a = gu.encode_docs(fx, interner)
for label, extra in (("bench", {}), ("bigprops", {"props_capacity": 20000}), ("notight", "nt")):
    caps = bench.capacities(dict(fx["config"]))
    if extra == "nt":
        for k in ("lds_page_capacity", "lds_unsettled_capacity", "lds_page_heap_capacity", "lds_narrow_overlap"):
            caps.pop(k)
    else:
        caps.update(extra)
    mt = MergeTreeBatch(len(fx["docs"]), delta_log_capacity=0, **caps)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    print(label, "grown", mt.last_grown(), "peaks", mt.last_paged_peaks(), "status", mt.status().tolist())
    for i, doc in enumerate(fx["docs"][:2]):
        exp = gu.expected(doc, interner)
        rows, leaves = mt.get_segments(i)
        e = np.asarray(exp["segs"])
        bad = np.flatnonzero((rows != e).any(axis=1)) if rows.shape == e.shape else "shape"
        print(" ", label, i, "bad rows", bad if isinstance(bad, str) else len(bad))
