"""Multi-GPU sharding logic on CPU: shard bounds, and a
world_size-2 gloo run that packs per-rank shards and assembles the single
stream from exchanged shard totals, checked against the oracle on the whole
batch."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O
from capnp_amd import shard


def test_shard_by_words_balanced_and_contiguous():
    rng = np.random.default_rng(2)
    sizes = rng.integers(0, 1000, 1000)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for world in (1, 2, 3, 8):
        b = shard.shard_by_words(offs, world)
        assert b[0] == 0 and b[-1] == 1000 and all(x <= y for x, y in zip(b, b[1:]))
        per = [int(offs[b[r + 1]] - offs[b[r]]) for r in range(world)]
        assert max(per) - min(per) <= 2 * int(sizes.max())
    assert shard.shard_by_words(np.array([0], np.uint64), 4) == [0] * 5
    assert shard.shard_even(10, 4) == [0, 2, 5, 7, 10]
    assert shard.exclusive_offsets([3, 0, 5]) == [0, 3, 3, 8]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_shard_concat(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    import _dist_worker as W
    world = 2
    mp.spawn(W.pack_concat_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    words, offs = W.batch()
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    packed = np.concatenate([np.load(tmp_path / f"packed{r}.npy") for r in range(world)])
    assert packed.tobytes() == ref.tobytes()
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(world)]
    goffs = [np.load(tmp_path / f"offs{r}.npy") for r in range(world)]
    # rank r's offsets cover chunks [c0, c1] of the whole batch
    for r in range(world):
        c0, c1 = int(metas[r][0]), int(metas[r][1])
        assert np.array_equal(goffs[r], ref_offs[c0:c1 + 1])
        assert int(metas[r][3]) == len(ref)
        assert float(metas[r][4]) == 1.5  # max over ranks of 0.5 + rank
