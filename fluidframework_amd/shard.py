"""Multi-GPU plumbing (one process per GPU): contiguous document shards and the single
collective of the replay path -- an all-gather of per-document checksums over RCCL/xGMI
(SURVEY.md 8e).  Documents are independent, so replay itself exchanges nothing."""
import numpy as np

from .wire import CHECKSUM_DTYPE


def shard_range(n_docs_total, world, rank):
    """Contiguous [lo, hi) of documents owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_docs_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_checksums(local, dist, device=None):
    """All-gathers every rank's mt_checksum array (equal shard sizes) and returns the
    concatenation in rank order.  `local` is either a numpy CHECKSUM_DTYPE array or a uint8
    torch tensor already holding the records (e.g. filled on the GPU by
    MergeTreeBatch.checksums_device)."""
    import torch
    if isinstance(local, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(local).view(np.uint8).copy())
        if device is not None:
            t = t.to(device)
    else:
        t = local
    world = dist.get_world_size()
    if dist.get_backend() == "nccl":
        out = torch.empty(world * t.numel(), dtype=torch.uint8, device=t.device)
        dist.all_gather_into_tensor(out, t)
    else:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        out = torch.cat(parts)
    return out.cpu().numpy().view(CHECKSUM_DTYPE)


def digest(sums):
    """Order-sensitive 64-bit digest of a checksum array (for logs)."""
    words = np.ascontiguousarray(sums).view(np.uint64)
    h = np.uint64(1469598103934665603)
    for i, w in enumerate(words):
        h = np.uint64((int(h) ^ int(w) ^ i) * 1099511628211 % (1 << 64))
    return int(h)
