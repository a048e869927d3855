"""Debug aid (GPU box, MT_PROF build): section time breakdown of one replay step.
    MT_EXTRA_FLAGS=-DMT_PROF MT_OUT=fluidframework_amd/libmtreplay_prof.so python fluidframework_amd/build.py --force
    MT_LIB_PATH=fluidframework_amd/libmtreplay_prof.so python profiles/tools/sections.py c3 10000 12500 [skew]
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd import MergeTreeBatch, _native  # noqa: E402

cfg = json.load(open("bench/configs.json"))[sys.argv[1]]
cfg = dict(cfg, ops=int(sys.argv[2]))
docs = int(sys.argv[3])
import bench  # noqa: E402
caps = bench.capacities(cfg)
if len(sys.argv) > 4 and sys.argv[4] == "skew":   # the c3skew class capacities for this length
    import bench_skew  # noqa: E402
    caps = bench_skew.class_caps(bench, cfg, cfg["ops"])
mt = MergeTreeBatch(docs, **caps)
b = mt.generate(cfg)
print("generation peaks", mt.last_paged_peaks())
seed_off, seed = mt.generated_seeds(cfg)
mt.load_initial_text(seed_off, seed)
out = np.zeros(128, dtype=np.uint64)
mt.lib.mt_debug_prof(mt.h, None, 1)
b.apply_async()
mt.sync()
print("kernel ms", mt.last_kernel_ms(), "hbm", mt.last_hbm_docs(), "peaks", mt.last_paged_peaks())
mt.lib.mt_debug_prof(mt.h, _native.ptr(out), 0)
# paged documents reuse slots 2, 4, 5 for pg_zamboni internals (scour_range, locate, heap pop)
names = ["split_seg", "boundary", "scour|pg_scour", "pack", "zamboni|pg_locate", "text_gc|pg_heap_pop", "op_insert", "op_range", "obs_prefix",
         "pg_views", "pg_win_load", "pg_win_flush", "pg_zamboni", "pg_find", "pg_pack1", "pg_apply_op"]
ops = docs * cfg["ops"]
# slots: engine 0..8, paged driver 9..15, MT_PROF2 finer engine timers 26..32, paged sub-timers 33..
names += [""] * (64 - len(names))
for k, n in {26: "scour need_nl", 27: "scour text merge", 28: "scour compaction", 29: "flat zamboni find",
             30: "insert split pass", 31: "(p2 14)", 32: "insert seg shift", 33: "flush purge",
             34: "flush table add", 35: "flush write page", 36: "pg_views table"}.items():
    names[k] = n
for i, n in enumerate(names):
    if n and out[64 + i]:
        print(f"{n:20s} ticks/op {out[i] / ops:10.1f}  calls/op {out[64 + i] / ops:8.3f}  ticks/call {out[i] / max(out[64 + i], 1):10.1f}")
# event counts (mt_paged.h PG_CNT)
events = {16: "zamboni heap pops", 17: "  pops of a gone id (0)", 18: "  pops switching the window",
          19: "  pops whose segment is gone", 20: "  pops of a scoured block (skip)", 21: "  scours",
          22: "  level-1 packs after a scour", 23: "window flushes writing slots", 24: "op window switches",
          25: "page splits"}
for k, n in events.items():
    print(f"{n:34s} per op {out[64 + k] / ops:8.4f}")
