"""Debug aid (GPU box): finds the shortest prefix of one document's op stream after which a
GPU tier's state differs from the oracle's (each trial = fresh document + one batch, so state
kept inside a launch is exercised).

    python tests/debug_bisect.py fixture ref_c2 1 '{"lds_seg_capacity": -1, "page_capacity": 256}'
    python tests/debug_bisect.py gen c3 3000 2 '{...}'
"""
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

if sys.argv[1] == "fixture":
    import golden_util as gu
    fx = gu.load(sys.argv[2])
    doc = int(sys.argv[3])
    a = gu.encode_docs(fx, gu.interner_for(fx), docs=[fx["docs"][doc]])
    seed = a["seed"][a["seed_off"][0]:a["seed_off"][1]]
    ops, text, props = a["ops"], a["text"], a["props"]
    opts = json.loads(sys.argv[4]) if len(sys.argv) > 4 else {}
else:
    cfg = json.load(open("bench/configs.json"))[sys.argv[2]]
    cfg = dict(cfg, ops=int(sys.argv[3]))
    g = pyoracle.generate(cfg, int(sys.argv[4]))
    seed, ops, text, props = g["seed"], g["ops"], g["text"], g["props"]
    opts = json.loads(sys.argv[5]) if len(sys.argv) > 5 else {}

opts.setdefault("seg_capacity", 4096)
opts.setdefault("text_capacity", 1 << 16)
opts.setdefault("delta_log_capacity", 1 << 18)
mt = MergeTreeBatch(1, **opts)
seed_off = np.array([0, len(seed)], dtype=np.int64)


def state_gpu(k):
    mt.load_initial_text(seed_off, seed)
    mt.apply_arrays(dict(ops=ops[:k], doc_off=np.array([0, k], dtype=np.int64), text=text, props=props))
    rows, leaves = mt.get_segments(0)
    return int(mt.status()[0]), rows, list(leaves), mt.get_text(0)


def state_oracle(k):
    od = pyoracle.OracleDoc.new(seed)
    od.apply_all(ops[:k], text, props)
    o = od.outputs()
    return 0, o["segs"], list(o["leaves"]), o["text"]


def same(k):
    g, o = state_gpu(k), state_oracle(k)
    return g[0] == o[0] and g[1].shape == o[1].shape and np.array_equal(g[1], o[1]) and g[2] == o[2] and g[3] == o[3]


n = len(ops)
if same(n):
    print("all", n, "ops equal")
    sys.exit(0)
lo, hi = 0, n          # same(lo) holds, same(hi) fails
while hi - lo > 1:
    mid = (lo + hi) // 2
    if same(mid):
        lo = mid
    else:
        hi = mid
print("first bad prefix", hi, "op", ops[hi - 1])
g, o = state_gpu(hi), state_oracle(hi)
print("status", g[0], "diag", mt.debug_raw(0)[1][27])
print("gpu leaves", g[2])
print("ora leaves", o[2])
print("gpu segs", [tuple(r[:4]) for r in g[1].tolist()])
print("ora segs", [tuple(r[:4]) for r in o[1].tolist()])
gl, ol = state_gpu(hi - 1), state_oracle(hi - 1)
print("before: leaves", gl[2])
print("before: segs", [tuple(r[:4]) for r in gl[1].tolist()])
