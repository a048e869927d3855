"""Debug aid (GPU box): the C5 end-to-end path (summary JSON -> MergeTreeBatch.catch_up ->
tails) against the device-only path (extracted records -> load) on a few documents: which
checksum fields differ, before and after the tails."""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402
from fluidframework_amd.snapdec import SummaryDecoder  # noqa: E402
from fluidframework_amd.snapshot import encode_chunks, load_arrays_from_extract, record_specs  # noqa: E402
from fluidframework_amd.wire import Interner  # noqa: E402

cfg = json.load(open("bench/configs.json"))["c5"]
docs, K, tail = 64, cfg["ops"], cfg["tail"]
caps = dict(seg_capacity=1024, text_capacity=1 << 14, heap_capacity=1024, props_capacity=1024, lds_seg_capacity=256)
mt = MergeTreeBatch(docs, **caps)
g1 = mt.generate(dict(cfg, ops=K))
counts, recs, text, props, mn, cu = mt.extract_snapshots_raw()
load = load_arrays_from_extract(counts, recs, text, props, mn, cu, cfg["chunk"])
g2 = mt.generate(dict(cfg, ops=K + tail))
host = g2.download()
idx = (np.arange(docs)[:, None] * (K + tail) + K + np.arange(tail)[None, :]).ravel()
tail_arr = dict(ops=host["ops"][idx], doc_off=np.arange(docs + 1, dtype=np.int64) * tail, text=host["text"],
                props=host["props"])
a = MergeTreeBatch(docs, **caps)
a.load_snapshots(load)
s_a0 = a.checksums()
it = Interner(synthetic=True)
c = np.asarray(counts, dtype=np.int64)
r0 = np.concatenate([[0], np.cumsum(c[:, 0])])
t0 = np.concatenate([[0], np.cumsum(c[:, 1])])
p0 = np.concatenate([[0], np.cumsum(c[:, 2])])
names = {i: f"client-{i}" for i in range(-2, 4096)}
summ = []
for d in range(docs):
    specs, lengths = record_specs(recs[r0[d]:r0[d + 1]], text[t0[d]:t0[d + 1]], props[p0[d]:p0[d + 1]], it, names)
    summ.append(encode_chunks(specs, lengths, int(mn[d]), int(cu[d]), cfg["chunk"]))
b = MergeTreeBatch(docs, **caps)
catchup, clients = b.catch_up(summ, Interner(synthetic=True), threads=4, slice_docs=16)
s_b0 = b.checksums()
for f in s_a0.dtype.names:
    print("after load", f, int((s_a0[f] != s_b0[f]).sum()), "docs differ")
print("status", a.status()[:8], b.status()[:8])
print("clients[0]", clients[0])
la, _, _ = SummaryDecoder(Interner(synthetic=True), 2).decode_packed_full(*SummaryDecoder.pack(summ[:1]))
l0 = {k: (v[: load["doc_off"][1]] if k == "segs" else v) for k, v in load.items()}
print("segs equal (doc 0)", np.array_equal(la["segs"], load["segs"][: load["doc_off"][1]]),
      la["segs"][:3], load["segs"][:3])
