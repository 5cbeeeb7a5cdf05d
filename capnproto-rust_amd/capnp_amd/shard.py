"""Multi-GPU sharding of a packed-codec batch.

Chunks are independent, so a batch shards into contiguous chunk ranges, one
per rank, with no collective on the data path.  Each rank packs its range into
its own buffer with its own offsets.  A single output stream is the in-order
concatenation of the shards: rank r's bytes start at the exclusive scan of
the shard totals.  The only collectives here are measurement and assembly
bookkeeping (a max of elapsed times, an all-gather of per-rank totals).

Works with any torch.distributed backend (nccl = RCCL on the GPU box, gloo on
CPU for the tests).
"""
import numpy as np


def shard_by_words(chunk_word_off, world):
    """Contiguous chunk ranges balanced by words: rank r gets chunks
    [bounds[r], bounds[r+1]).  chunk_word_off: n+1 non-decreasing offsets."""
    off = np.asarray(chunk_word_off, dtype=np.uint64)
    n = len(off) - 1
    if world <= 0:
        raise ValueError("world must be positive")
    if n <= 0:
        return [0] * (world + 1)
    base, total = int(off[0]), int(off[-1] - off[0])
    targets = [base + (total * r) // world for r in range(world + 1)]
    bounds = [int(np.searchsorted(off[:-1], t, side="left")) for t in targets]
    bounds[0], bounds[-1] = 0, n
    for r in range(1, world + 1):  # monotone
        bounds[r] = max(bounds[r], bounds[r - 1])
    return bounds


def shard_even(nchunks, world):
    """Contiguous, equal-count chunk ranges (chunks of equal size)."""
    return [(nchunks * r) // world for r in range(world + 1)]


def exclusive_offsets(totals):
    """Start of each shard in the concatenated stream, plus the total."""
    out = [0]
    for t in totals:
        out.append(out[-1] + int(t))
    return out


def gather_totals(total, group=None, device=None):
    """All-gather one integer per rank (the shard's packed size)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.tensor([int(total)], dtype=torch.int64, device=device)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [int(o.item()) for o in outs]


def max_over_ranks(value, group=None, device=None):
    """Max of a float over ranks (the bench's timed-region length)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def global_chunk_offsets(local_out_off, shard_start):
    """Rank-local packed offsets (n_r + 1, starting at 0) shifted to the
    concatenated stream; drops the local end marker except on the last rank."""
    return np.asarray(local_out_off, dtype=np.uint64) + np.uint64(shard_start)
