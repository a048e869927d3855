"""Debug aid (GPU box): replays one synthetic document op by op on the GPU (one-op batches)
and on the oracle, and reports the first op after which the segment tables differ.

    python tests/debug_step.py c2 400 [doc] [lds_seg_capacity]
"""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(0, ".")
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

cfg = json.load(open("bench/configs.json"))[sys.argv[1]]
cfg = dict(cfg, ops=int(sys.argv[2]))
doc = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lds = int(sys.argv[4]) if len(sys.argv) > 4 else 0
g = pyoracle.generate(cfg, doc)
od = pyoracle.OracleDoc.new(g["seed"])
mt = MergeTreeBatch(1, seg_capacity=4096, text_capacity=1 << 16, lds_seg_capacity=lds, delta_log_capacity=1 << 16)
seed_off = np.array([0, len(g["seed"])], dtype=np.int64)
mt.load_initial_text(seed_off, g["seed"])
L = pyoracle.lib()
ops = g["ops"]


def ostate():
    o = od.outputs()
    return o["segs"], o["leaves"], o["text"]


for i in range(len(ops)):
    before = (mt.get_segments(0), ostate())
    L.orc_apply(od.h, ctypes.c_void_p(ops.ctypes.data + 32 * i), pyoracle._p(g["text"]), pyoracle._p(g["props"]))
    mt.apply_arrays(dict(ops=ops[i:i + 1], doc_off=np.array([0, 1], dtype=np.int64), text=g["text"],
                         props=g["props"]))
    rows, leaves = mt.get_segments(0)
    osegs, oleaves, otext = ostate()
    st = int(mt.status()[0])
    same = st == 0 and rows.shape == osegs.shape and np.array_equal(rows, osegs) and list(leaves) == list(oleaves)
    if same:
        same = mt.get_text(0) == otext
    if not same:
        print("first divergence after op", i, ops[i], "status", st)
        print("gpu before:", before[0][0].tolist(), list(before[0][1]))
        print("ora before:", before[1][0].tolist(), before[1][1])
        print("gpu after:", rows.tolist(), list(leaves))
        print("ora after:", osegs.tolist(), oleaves)
        print("gpu text:", repr(mt.get_text(0)))
        print("ora text:", repr(otext))
        dl = list(mt.get_delta_log(0))
        k = max(i for i in range(len(dl)) if dl[i] == 0x7777 and i + 5 < len(dl) and dl[i + 1] == ops[i if False else 0]["pos1"] * 0 + int(ops[i]["pos1"])) if False else None
        idx = [j for j in range(len(dl)) if dl[j] == 0x7777]
        for j in idx[-3:]:
            print("dbg", dl[j:j + 5 + 64])
        break
else:
    print("all", len(ops), "ops equal")
