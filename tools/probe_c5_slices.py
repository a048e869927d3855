"""Probe (GPU box): where a C5 catch-up slice's time goes -- native decode, host->device upload
(mt_snapshots_upload_range), device load -- for synthetic bench-shaped summaries."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd import MergeTreeBatch  # noqa: E402
from fluidframework_amd.snapdec import SummaryDecoder  # noqa: E402
from fluidframework_amd.snapshot import encode_chunks, record_specs  # noqa: E402
from fluidframework_amd.wire import Interner  # noqa: E402

cfg = json.load(open("bench/configs.json"))["c5"]
n_emit, S = 2000, 16384
caps = dict(seg_capacity=1024, text_capacity=1 << 14, heap_capacity=1024, props_capacity=1024, lds_seg_capacity=256)
mt = MergeTreeBatch(n_emit, **caps)
mt.generate(dict(cfg, ops=cfg["ops"]))
counts, recs, text, props, mn, cu = mt.extract_snapshots_raw()
it = Interner(synthetic=True)
c = np.asarray(counts, dtype=np.int64)
r0, t0, p0 = (np.concatenate([[0], np.cumsum(c[:, k])]) for k in range(3))
names = {i: f"client-{i}" for i in range(-2, 4096)}
em = []
for d in range(n_emit):
    sp, ln = record_specs(recs[r0[d]:r0[d + 1]], text[t0[d]:t0[d + 1]], props[p0[d]:p0[d + 1]], it, names)
    em.append(SummaryDecoder.pack([encode_chunks(sp, ln, int(mn[d]), int(cu[d]), cfg["chunk"])]))
paths = [em[d % n_emit][0][0] for d in range(S)]
blobs = [em[d % n_emit][1][0] for d in range(S)]
off = list(range(S + 1))
big = MergeTreeBatch(S, **caps)
for th in (16, 15, 8):
    dec = SummaryDecoder(Interner(synthetic=True), th)
    for rep in range(3):
        t = time.perf_counter()
        out, _, _ = dec.decode_packed_full(paths, blobs, off)
        t1 = time.perf_counter()
        s = big.upload_snapshots(out)
        t2 = time.perf_counter()
        s.load_async()
        big.sync()
        t3 = time.perf_counter()
        s.free()
        t4 = time.perf_counter()
        nb = out["segs"].nbytes + out["text"].nbytes + out["props"].nbytes
        print(f"threads {th}: decode {1e3*(t1-t):.1f} ms, upload {1e3*(t2-t1):.1f} ms ({nb/1e6:.0f} MB), "
              f"load {1e3*(t3-t2):.1f} ms, free {1e3*(t4-t3):.1f} ms for {S} docs")
# the pipelined catch-up itself (decode into page-locked arenas, upload, load)
for sl in (4096, 16384):
    for rep in range(2):
        t = time.perf_counter()
        big.catch_up(None, Interner(synthetic=True), threads=16, slice_docs=sl, packed=(paths, blobs, off))
        print(f"catch_up slice {sl}: {1e3*(time.perf_counter()-t):.1f} ms for {S} docs")
