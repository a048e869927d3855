"""Replays a fixture on one storage tier and prints each document's status and header
diagnostics (status, cap_cause, n_seg, heap_n, props_top, next_uid).
    python tools/debug_wide.py ref_wide lds"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import golden_util as gu  # noqa: E402
from test_gpu_parity import TIERS, _gpu_batch  # noqa: E402


def main():
    name, tier = sys.argv[1], sys.argv[2]
    fx = gu.load(name)
    it = gu.interner_for(fx)
    a = gu.encode_docs(fx, it)
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    st = mt.status()
    for d in range(len(fx["docs"])):
        rows, hdr = mt.debug_raw(d)
        print(d, "status", st[d], "diag", hdr[27], "n_seg", hdr[0], "heap_n", hdr[2], "cur_seq", hdr[3],
              "min_seq", hdr[4], "props_top", hdr[7], "next_uid", hdr[9], flush=True)


if __name__ == "__main__":
    main()
