"""Debug aid: compare per-op writer view lengths of the GPU generator vs the oracle."""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

cfg = json.load(open("bench/configs.json"))[sys.argv[1]]
cfg = dict(cfg, ops=int(sys.argv[2]))
docs = int(sys.argv[3])
mt = MergeTreeBatch(docs, seg_capacity=4096)
tr = np.zeros(docs * cfg["ops"], dtype=np.int32)
b = mt.generate(cfg, trace=tr)
got = b.download()
L = pyoracle.lib()
L.orc_set_gen_trace.argtypes = [ctypes.c_void_p]
for d in range(docs):
    otr = np.zeros(cfg["ops"], dtype=np.int32)
    L.orc_set_gen_trace(otr.ctypes.data_as(ctypes.c_void_p))
    g = pyoracle.generate(cfg, d)
    L.orc_set_gen_trace(None)
    gt = tr[d * cfg["ops"]:(d + 1) * cfg["ops"]]
    diff = np.nonzero(gt != otr)[0]
    if len(diff):
        k = diff[0]
        print("doc", d, "first view-length diff at op", k + 1, "gpu", gt[k], "oracle", otr[k])
        lo = got["doc_off"][d]
        print(" gpu ops around:", got["ops"][lo + max(0, k - 3): lo + k + 1])
        print(" ora ops around:", g["ops"][max(0, k - 3): k + 1])
    else:
        print("doc", d, "view lengths equal")
