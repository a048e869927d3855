"""Ingest pipeline probe (GPU box): bench.ingest_pipeline at several encoder thread counts,
one line each (overlapped rate, stage rates, fraction of the slowest, per-slice encode s).
    python tools/ingest_probe.py 16 15 14"""
import gzip
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fluidframework_amd.opdec import MessageDecoder  # noqa: E402
from fluidframework_amd.wire import compact_msgs_to_dicts  # noqa: E402

fx = json.load(gzip.open(os.path.join(bench.REPO, "tests", "golden", "ref_c3_full.json.gz"), "rt"))
blobs = MessageDecoder.pack([compact_msgs_to_dicts(d["msgs"]) for d in fx["docs"]])
caps = bench.capacities(json.load(open(os.path.join(bench.REPO, "bench", "configs.json")))["c3"])
print("host cores", bench.host_cores(), flush=True)
for th in [int(x) for x in sys.argv[1:]]:
    p = bench.ingest_pipeline(caps, 0, fx, blobs, th)
    print(th, round(p["value"] / 1e6, 2), {k: round(v / 1e6, 2) for k, v in p["stage_rates"].items()},
          p["fraction_of_slowest"], p["busy_s"], p["encode_slices_s"], p["checksums_equal_oracle"], flush=True)
