"""Debug aid (GPU box): generate a config on the GPU, replay it, compare per-document
checksums with the oracle and list the mismatching documents and fields.

    python tests/debug_find.py c2 2000 1000 [lds_seg_capacity]
"""
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(0, ".")
import pyoracle  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

cfg = json.load(open("bench/configs.json"))[sys.argv[1]]
cfg = dict(cfg, ops=int(sys.argv[2]))
docs = int(sys.argv[3])
lds = int(sys.argv[4]) if len(sys.argv) > 4 else 0
mt = MergeTreeBatch(docs, seg_capacity=512, text_capacity=1 << 15, heap_capacity=1024,
                    props_capacity=640, lds_seg_capacity=lds)
b = mt.generate(cfg)
gsums = mt.checksums()
host = b.download()
seed_off, seed = mt.generated_seeds(cfg)
mt.load_initial_text(seed_off, seed)
b.apply_async()
mt.sync()
print("hbm docs", mt.last_hbm_docs())
sums = mt.checksums()
osums, ost = pyoracle.replay_batch(dict(host, seed_off=seed_off, seed=seed), threads=8)
bad = np.nonzero(osums != sums)[0]
print("mismatching docs:", len(bad), bad[:20].tolist(), "gen==replay", bool(np.array_equal(gsums, sums)))
for d in bad[:5]:
    print(d, {f: (int(sums[d][f]), int(osums[d][f])) for f in sums.dtype.names if sums[d][f] != osums[d][f]})
