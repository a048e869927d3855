"""N > 1 path on CPU (gloo, world size 2): contiguous document shards and the checksum
all-gather reproduce the single-process result.  Checksums come from the oracle here (the
test exercises the host sharding/collective logic; the GPU path is covered by -m gpu)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fluidframework_amd.shard import digest, gather_checksums, shard_range
from fluidframework_amd.wire import CHECKSUM_DTYPE

DOCS, OPS = 6, 120


def _cfg():
    import json
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return dict(json.load(open(os.path.join(repo, "bench", "configs.json")))["c3"], ops=OPS)


def _doc_sums(lo, hi):
    import pyoracle
    out = np.zeros(hi - lo, dtype=CHECKSUM_DTYPE)
    for i, d in enumerate(range(lo, hi)):
        g = pyoracle.generate(_cfg(), d, keep=True)
        out[i] = g["doc"].outputs()["checksum"]
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(DOCS, world, rank)
    got = gather_checksums(_doc_sums(lo, hi), dist)
    if rank == 0:
        q.put(got.tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_ranges_cover_every_document_once():
    for n in (0, 1, 7, 100):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_gloo_world2_checksum_allgather_equals_single_process(oracle_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=300), dtype=CHECKSUM_DTYPE)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _doc_sums(0, DOCS)
    assert np.array_equal(got, ref)
    assert digest(got) == digest(ref)
