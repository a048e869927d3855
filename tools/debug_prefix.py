"""Debug aid (not a test): replay every prefix of one fixture document on the GPU (one
document per prefix, one launch) and report the first op after which the GPU state differs
from the CPU oracle.  Usage: python tests/debug_prefix.py <fixture> <doc>"""
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
import golden_util as gu  # noqa: E402
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

name, di = sys.argv[1], int(sys.argv[2])
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
hi_cap = int(sys.argv[4]) if len(sys.argv) > 4 else 10 ** 9
fx = gu.load(name)
interner = gu.interner_for(fx)
doc = fx["docs"][di]
a = gu.encode_docs(fx, interner, [doc])
n = len(a["ops"])
hi = min(n, hi_cap)
ks = list(range(lo, hi + 1))
seed = a["seed"][: a["seed_off"][1]]
mt = MergeTreeBatch(len(ks), seg_capacity=4096, delta_log_capacity=0)
seed_off = np.arange(len(ks) + 1, dtype=np.int64) * len(seed)
mt.load_initial_text(seed_off, np.tile(seed, len(ks)))
idx = np.concatenate([np.arange(k) for k in ks]) if ks else np.zeros(0, int)
off = np.zeros(len(ks) + 1, dtype=np.int64)
off[1:] = np.cumsum(ks)
mt.apply_arrays(dict(a, ops=a["ops"][idx], doc_off=off))
st = mt.status()
od = pyoracle.OracleDoc.new(seed)
L = pyoracle.lib()
text, props = np.ascontiguousarray(a["text"]), np.ascontiguousarray(a["props"])
ops = np.ascontiguousarray(a["ops"])
for j, k in enumerate(ks):
    if k > 0:
        L.orc_apply(od.h, pyoracle.ctypes.c_void_p(ops.ctypes.data + 32 * (k - 1)), pyoracle._p(text), pyoracle._p(props))
    if k < lo:
        continue
    o = od.outputs()
    rows, leaves = mt.get_segments(j)
    g_text = mt.get_text(j)
    bad = []
    if st[j]:
        bad.append(f"status {st[j]}")
    if rows.tolist() != o["segs"].tolist():
        bad.append("segs")
    if leaves != o["leaves"]:
        bad.append("leaves")
    if g_text != o["text"]:
        bad.append("text")
    if bad:
        print("first divergence after op", k, bad)
        print("op", ops[k - 1] if k else None)
        print("oracle leaves", o["leaves"])
        print("gpu    leaves", leaves)
        og, gg = o["segs"].tolist(), rows.tolist()
        for i in range(max(len(og), len(gg))):
            x = og[i] if i < len(og) else None
            y = gg[i] if i < len(gg) else None
            if x != y:
                print(" seg", i, "oracle", x, "gpu", y)
        break
else:
    print("no divergence in", lo, "..", hi)
