"""Debug aid (GPU box, MT_PROF build): section time breakdown of one C2 replay step.
    MT_EXTRA_FLAGS=-DMT_PROF python fluidframework_amd/build.py --force   (here)
    python tests/debug_prof.py c2 2000 10000
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd import MergeTreeBatch, _native  # noqa: E402

cfg = json.load(open("bench/configs.json"))[sys.argv[1]]
cfg = dict(cfg, ops=int(sys.argv[2]))
docs = int(sys.argv[3])
mt = MergeTreeBatch(docs, seg_capacity=512, text_capacity=1 << 15, heap_capacity=1024, props_capacity=640)
b = mt.generate(cfg)
seed_off, seed = mt.generated_seeds(cfg)
mt.load_initial_text(seed_off, seed)
out = np.zeros(32, dtype=np.uint64)
mt.lib.mt_debug_prof(mt.h, None, 1)
b.apply_async()
mt.sync()
print("kernel ms", mt.last_kernel_ms(), "hbm", mt.last_hbm_docs())
mt.lib.mt_debug_prof(mt.h, _native.ptr(out), 0)
names = ["split_seg", "boundary", "scour_block", "pack", "zamboni", "text_gc", "op_insert", "op_range", "obs_prefix"]
ops = docs * cfg["ops"]
for i, n in enumerate(names):
    print(f"{n:12s} ticks/op {out[i] / ops:10.1f}  calls/op {out[16 + i] / ops:8.3f}  ticks/call {out[i] / max(out[16 + i], 1):10.1f}")
