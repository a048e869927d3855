"""Multi-GPU plumbing (one process per GPU): contiguous document shards and the single
collective of the replay path -- an all-gather of per-document checksums over RCCL/xGMI
(SURVEY.md 8e).  Documents are independent, so replay itself exchanges nothing."""
import numpy as np

from .wire import CHECKSUM_DTYPE

REC = CHECKSUM_DTYPE.itemsize


def shard_range(n_docs_total, world, rank):
    """Contiguous [lo, hi) of documents owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_docs_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def padded_shard(n_docs_total, world):
    """Records per rank in the all-gather buffer: the largest shard (ceil(n / world))."""
    return -(-n_docs_total // world) if world else 0


def gather_checksums(local, dist, device=None, n_total=None):
    """All-gathers every rank's mt_checksum array and returns the concatenation in rank
    order.  `local` is either a numpy CHECKSUM_DTYPE array or a uint8 torch tensor already
    holding the records (e.g. filled on the GPU by MergeTreeBatch.checksums_device).

    Collectives need equal sizes: with `n_total` given, every rank's records are padded to
    padded_shard(n_total, world) and the padding is dropped again with shard_range, so
    shards that differ by one (n_total not divisible by the world size) gather correctly.
    Without it every rank must pass the same number of records."""
    import torch
    world = dist.get_world_size()
    if isinstance(local, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(local, dtype=CHECKSUM_DTYPE).view(np.uint8).copy())
        if device is not None:
            t = t.to(device)
    else:
        t = local
    n_local = t.numel() // REC
    per = padded_shard(n_total, world) if n_total is not None else n_local
    if n_total is not None:
        lo, hi = shard_range(n_total, world, dist.get_rank())
        if hi - lo != n_local:
            raise ValueError(f"rank {dist.get_rank()} holds {n_local} records, its shard is {hi - lo}")
    elif dist.get_backend() != "nccl":
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([n_local], dtype=torch.int64))
        if any(int(s) != n_local for s in sizes):
            raise ValueError("unequal shard sizes: pass n_total")
    if per != n_local:
        pad = torch.zeros((per - n_local) * REC, dtype=torch.uint8, device=t.device)
        t = torch.cat([t.reshape(-1), pad])
    if dist.get_backend() == "nccl":
        out = torch.empty(world * per * REC, dtype=torch.uint8, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous())
    else:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t.contiguous())
        out = torch.cat(parts)
    recs = out.cpu().numpy().view(CHECKSUM_DTYPE)
    if n_total is None or per * world == n_total:
        return recs
    keep = [recs[r * per: r * per + (hi - lo)] for r, (lo, hi) in
            ((r, shard_range(n_total, world, r)) for r in range(world))]
    return np.concatenate(keep)


def digest(sums):
    """Order-sensitive 64-bit digest of a checksum array (for logs)."""
    words = np.ascontiguousarray(sums).view(np.uint64)
    h = np.uint64(1469598103934665603)
    for i, w in enumerate(words):
        h = np.uint64((int(h) ^ int(w) ^ i) * 1099511628211 % (1 << 64))
    return int(h)
