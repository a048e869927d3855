"""Debug aid: GPU-generate a few ops, then compare GPU state to the oracle replaying the
GPU-generated ops, and the GPU's generation-time view lengths to the oracle's."""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

cfg = json.load(open("bench/configs.json"))["c2"]
ops_n = int(sys.argv[1])
cfg = dict(cfg, ops=ops_n)
docs = 4
mt = MergeTreeBatch(docs, seg_capacity=4096)
tr = np.zeros(docs * ops_n * 4, dtype=np.int32)
b = mt.generate(cfg, trace=tr)
got = b.download()
seed_off, seed = mt.generated_seeds(cfg)
for d in range(docs):
    lo, hi = got["doc_off"][d], got["doc_off"][d + 1]
    od = pyoracle.OracleDoc.new(seed[seed_off[d]:seed_off[d + 1]])
    ops = np.ascontiguousarray(got["ops"][lo:hi])
    L = pyoracle.lib()
    txt = np.ascontiguousarray(got["text"])
    prp = np.ascontiguousarray(got["props"])
    olens = []
    for k in range(hi - lo):
        olens.append(L.orc_view_length(od.h, int(ops[k]["ref_seq"]), int(ops[k]["client"])))
        L.orc_apply(od.h, ctypes.c_void_p(ops.ctypes.data + 32 * k), pyoracle._p(txt), pyoracle._p(prp))
    o = od.outputs()
    rows, leaves = mt.get_segments(d)
    print("doc", d, "state equal:", rows.tolist() == o["segs"].tolist(), "text equal:", mt.get_text(d) == o["text"])
    print("   gpu trace  ", tr.reshape(docs, ops_n, 4)[d].tolist())
    print("   oracle lens", olens)
    if rows.tolist() != o["segs"].tolist():
        print("   gpu segs", rows.tolist())
        print("   ora segs", o["segs"].tolist())
        print("   ops", ops.tolist())
# dump GPU segments after generation and evaluate the view formula in Python
for d in range(docs):
    rows, leaves = mt.get_segments(d)
    print("doc", d, "rows", rows.tolist())
