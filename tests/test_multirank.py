"""N > 1 path on CPU (gloo, world size 2): contiguous document shards, the checksum
all-gather (including shards of unequal size) and bench.py's own rank code -- the
verify_shards step every rank runs after the timed region -- reproduce the single-process
result and catch a corrupted shard.  Checksums come from the oracle here (the test
exercises the host sharding / collective / verification logic; the GPU path is covered by
-m gpu)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fluidframework_amd.shard import digest, gather_checksums, padded_shard, shard_range
from fluidframework_amd.wire import CHECKSUM_DTYPE

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS, OPS = 5, 120          # 5 documents over 2 ranks: shards of 3 and 2


def _cfg():
    import json
    return dict(json.load(open(os.path.join(REPO, "bench", "configs.json")))["c3"], ops=OPS)


def _doc_sums(lo, hi):
    import pyoracle
    out = np.zeros(hi - lo, dtype=CHECKSUM_DTYPE)
    for i, d in enumerate(range(lo, hi)):
        g = pyoracle.generate(_cfg(), d, keep=True)
        out[i] = g["doc"].outputs()["checksum"]
    return out


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _gather_worker(rank, world, port, q):
    _init(rank, world, port)
    lo, hi = shard_range(DOCS, world, rank)
    got = gather_checksums(_doc_sums(lo, hi), dist, n_total=DOCS)
    if rank == 0:
        q.put(got.tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _bench_worker(rank, world, port, q, corrupt_rank):
    """bench.py's post-timing rank code with oracle checksums standing in for the device's."""
    _init(rank, world, port)
    import bench
    per = 3
    cfg = _cfg()
    local = _doc_sums(rank * per, (rank + 1) * per)
    gen = local.copy()
    if rank == corrupt_rank:
        local[1]["text_hash"] ^= np.uint64(1)
    rep = bench.verify_shards(dist, rank, world, per * world, cfg, local, gen, None, per, 2)
    if rank == 0:
        q.put(rep)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, q) + args) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def test_shard_ranges_cover_every_document_once():
    for n in (0, 1, 7, 100):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) == padded_shard(n, w)


def test_gloo_world2_uneven_checksum_allgather_equals_single_process(oracle_lib):
    got = np.frombuffer(_run(_gather_worker), dtype=CHECKSUM_DTYPE)
    ref = _doc_sums(0, DOCS)
    assert np.array_equal(got, ref)
    assert digest(got) == digest(ref)


@pytest.mark.parametrize("corrupt_rank", [-1, 1])
def test_gloo_world2_bench_verify_shards(oracle_lib, corrupt_rank):
    rep = _run(_bench_worker, corrupt_rank)
    assert rep["docs_gathered"] == 6 and rep["oracle_docs"] == 6
    if corrupt_rank < 0:
        assert rep["replay_equals_generation"] and rep["oracle_mismatches"] == 0
    else:   # a wrong document on rank 1 is caught on rank 0 both ways
        assert not rep["replay_equals_generation"] and rep["oracle_mismatches"] == 1


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """`bench.py --gpus N` outside a launcher starts N ranks via torch.distributed.run (the
    child command is checked, nothing is run)."""
    import subprocess
    sys.path.insert(0, REPO)
    import bench
    seen = {}
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.update(cmd=cmd, env=env) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert bench.launch(bench.parse()) == 0
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
