"""Skewed batches on CPU (fluidframework_amd/skew.py): the c3skew length distribution, shards
balanced by message count -- including their use by world-size-2 gloo ranks, whose shards
cover the job once and whose all-gathered message counts agree -- and the size classes the
bench replays per handle."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fluidframework_amd.skew import shard_range_ops, size_classes, zipf_lengths

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_zipf_lengths_total_cap_and_seeded_order():
    a = zipf_lengths(100_000, 10 ** 9, 1.1, 200_000, 7)
    assert a.dtype == np.int32 and a.sum() == 10 ** 9
    assert a.max() == 200_000 and a.min() >= 1
    assert (a == 200_000).sum() > 1000           # the capped head
    assert np.median(a) < 5000                   # most documents are short
    b = zipf_lengths(100_000, 10 ** 9, 1.1, 200_000, 7)
    assert np.array_equal(a, b)
    c = zipf_lengths(100_000, 10 ** 9, 1.1, 200_000, 8)
    assert np.array_equal(np.sort(a), np.sort(c)) and not np.array_equal(a, c)
    assert np.argmax(a) != 0                     # long documents are scattered


def test_op_balanced_shards_cover_once_and_balance():
    lens = zipf_lengths(20_000, 10 ** 8, 1.1, 100_000, 3)
    for w in (1, 2, 3, 8):
        spans = [shard_range_ops(lens, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == len(lens)
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        ops = [int(lens[a:b].sum()) for a, b in spans]
        assert max(ops) - min(ops) <= 2 * int(lens.max())
        assert max(ops) <= lens.sum() / w + lens.max()
    assert shard_range_ops(np.zeros(0, np.int32), 2, 1) == (0, 0)
    # equal lengths: the same shards as by document count (up to one document)
    eq = np.full(10, 7, np.int32)
    assert [shard_range_ops(eq, 2, r) for r in range(2)] == [(0, 5), (5, 10)]


def test_size_classes_partition_longest_first():
    lens = zipf_lengths(20_000, 10 ** 8, 1.1, 100_000, 3)
    cls = size_classes(lens, [2000, 20_000, 100_000])
    assert [b for b, _ in cls] == sorted((b for b, _ in cls), reverse=True)
    idx = np.sort(np.concatenate([i for _, i in cls]))
    assert np.array_equal(idx, np.arange(len(lens)))
    for b, i in cls:
        assert lens[i].max() <= b


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = zipf_lengths(5000, 2 * 10 ** 7, 1.1, 50_000, 11)
    lo, hi = shard_range_ops(lens, world, rank)
    mine = torch.tensor([lo, hi, int(lens[lo:hi].sum())], dtype=torch.int64)
    parts = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        q.put([p.tolist() for p in parts])
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_op_balanced_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lens = zipf_lengths(5000, 2 * 10 ** 7, 1.1, 50_000, 11)
    (lo0, hi0, n0), (lo1, hi1, n1) = got
    assert lo0 == 0 and hi0 == lo1 and hi1 == len(lens)
    assert n0 + n1 == lens.sum()
    assert abs(n0 - n1) <= 2 * lens.max()
    # by document count the split would be far off balance for this skew
    half = len(lens) // 2
    assert abs(n0 - n1) < abs(int(lens[:half].sum()) - int(lens[half:].sum())) or abs(n0 - n1) <= lens.max()
