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
tcap = int(sys.argv[5]) if len(sys.argv) > 5 else 1 << 16
mt = MergeTreeBatch(1, seg_capacity=4096, text_capacity=tcap, lds_seg_capacity=lds, delta_log_capacity=1 << 16)
seed_off = np.array([0, len(g["seed"])], dtype=np.int64)
mt.load_initial_text(seed_off, g["seed"])
L = pyoracle.lib()
ops = g["ops"]


def ostate():
    o = od.outputs()
    return o["segs"], o["leaves"], o["text"]


for i in range(len(ops)):
    before = (mt.get_segments(0), ostate())
    raw_before = mt.debug_raw(0)
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
        print("gpu leaves before:", list(before[0][1]), "after", list(leaves))
        print("ora after:", [tuple(r[:2]) for r in osegs.tolist()], oleaves)
        print("gpu text:", repr(mt.get_text(0)))
        print("ora text:", repr(otext))
        rb, hb = raw_before
        ra, ha = mt.debug_raw(0)
        print("hdr before text_top/half", hb[5], hb[6], "after", ha[5], ha[6])
        print("raw before (len, off, w>>16, w&3):", [(int(r[0]), int(r[4]), int(r[7] >> 16), int(r[7] & 3)) for r in rb])
        print("raw after:", [(int(r[0]), int(r[4]), int(r[7] >> 16), int(r[7] & 3)) for r in ra])
        dl = list(mt.get_delta_log(0))
        k = max(i for i in range(len(dl)) if dl[i] == 0x7777 and i + 5 < len(dl) and dl[i + 1] == ops[i if False else 0]["pos1"] * 0 + int(ops[i]["pos1"])) if False else None
        idx = [j for j in range(len(dl)) if dl[j] == 0x7777]
        for j in idx[-3:]:
            print("dbg", dl[j:j + 5 + 64])
        break
else:
    print("all", len(ops), "ops equal")
