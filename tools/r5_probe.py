"""Probe: the ref_wide_long document on the paged / grow tiers -- status, diagnostic word,
growth and overlap arena (round-5 debugging of the overflow-set reclamation test)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import golden_util as gu
from fluidframework_amd import MergeTreeBatch

fx = gu.load("ref_wide_long")
interner = gu.interner_for(fx)
a = gu.encode_docs(fx, interner)
TIERS = {"paged": dict(lds_seg_capacity=-1, page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048),
         "grow": dict(lds_seg_capacity=16, page_capacity=12, unsettled_capacity=16, page_heap_capacity=16)}
for tier, caps in TIERS.items():
    for oa in (512, 0):
        kw = dict(caps, delta_log_capacity=1 << 21, seg_capacity=8192, text_capacity=1 << 17)
        if oa:
            kw["overlap_arena_capacity"] = oa
        mt = MergeTreeBatch(1, **kw)
        mt.load_initial_text(a["seed_off"], a["seed"])
        mt.apply_arrays(a)
        rows, hdr = mt.debug_raw(0)
        print(tier, oa, "status", int(mt.status()[0]), "diag", int(hdr[27]), "cur_seq", int(hdr[3]),
              "grown", mt.last_grown(), "arena", mt.get_overlap_arena(0), flush=True)
        mt.close()
