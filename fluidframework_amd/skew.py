"""Documents of unequal length (bench config c3skew; SURVEY.md section 7 hard part 5, 8e).

A real op log is skewed: a few documents carry most of the messages.  Three pieces serve it:

* `zipf_lengths` -- the synthetic workload: the C3 job's 10^9 messages spread over its 100k
  documents with Zipf-distributed lengths (rank r gets ~ r^-s, capped), assigned to documents
  in a seeded random order (long documents are scattered, not first).
* `shard_range_ops` -- contiguous shards balanced by message count rather than by documents.
* `size_classes` -- documents grouped by length; each class is replayed by its own handle,
  sized (LDS and HBM capacities) for its longest document, on its own HIP stream, the class
  of the longest documents launched first.  Inside a batch the library dispatches documents
  longest first by itself (mt_batch order, DevState.order).
"""
import numpy as np


def zipf_lengths(n_docs, total_ops, s, cap, seed):
    """int32[n_docs] message counts summing to total_ops: min(c r^-s, cap) for the document of
    rank r (c solved for the total), at least 1 each, ranks assigned by a seeded permutation."""
    if not n_docs <= total_ops <= n_docs * cap:
        raise ValueError(f"zipf_lengths: {total_ops} messages do not fit {n_docs} documents of 1..{cap}")
    r = np.arange(1, n_docs + 1, dtype=np.float64)
    lo, hi = 1.0, 1e18
    for _ in range(300):
        m = (lo * hi) ** 0.5
        if np.minimum(m * r ** -s, cap).sum() < total_ops:
            lo = m
        else:
            hi = m
    lens = np.maximum(np.floor(np.minimum(lo * r ** -s, cap)), 1).astype(np.int64)
    # the residual of the rounding, one message per document per pass (several passes when it
    # exceeds the documents still below the cap / above 1)
    while True:
        resid = int(total_ops - lens.sum())
        if resid > 0:
            free = np.flatnonzero(lens < cap)
            lens[free[:resid]] += 1
        elif resid < 0:
            lens[np.flatnonzero(lens > 1)[resid:]] -= 1
        else:
            break
    assert lens.sum() == total_ops
    perm = np.random.default_rng(seed).permutation(n_docs)
    out = np.empty(n_docs, dtype=np.int32)
    out[perm] = lens
    return out


def shard_range_ops(lens, world, rank):
    """Contiguous [lo, hi) of documents owned by `rank`, cut where the running message count
    crosses k / world of the total (each cut at the nearer document boundary), so the ranks'
    message counts differ by at most about one document's."""
    c = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    n = len(c) - 1

    def cut(k):
        if k <= 0:
            return 0
        if k >= world:
            return n
        t = c[-1] * k / world
        i = int(np.searchsorted(c, t, side="left"))
        if i > 0 and t - c[i - 1] < c[min(i, n)] - t:
            i -= 1
        return min(max(i, 0), n)

    lo, hi = cut(rank), cut(rank + 1)
    return lo, max(lo, hi)


def size_classes(lens, bounds):
    """[(max_ops, indices)] for the classes (0, b0], (b0, b1], ... of `bounds` (ascending; the
    last must cover max(lens)), longest class first, empty classes dropped."""
    lens = np.asarray(lens)
    if len(lens) and lens.max() > bounds[-1]:
        raise ValueError("size_classes: a document is longer than the last bound")
    out, lo = [], 0
    for b in bounds:
        idx = np.flatnonzero((lens > lo) & (lens <= b)) if lo else np.flatnonzero(lens <= b)
        if len(idx):
            out.append((int(b), idx))
        lo = b
    return out[::-1]
