"""Chunk-step pack (pack_cs_kernel, chunks_per_tile 16) over batches of
thousands of tiles that mix every tile kind: tiles with a chunk over 128
words (streaming size pass, bytes by pack_ovf_kernel), tiles whose packed
bytes overflow the staging regions (adversarial 0xFF / 6-byte words), empty
chunks and a short last tile.  Bytes, offsets and the record sync index must
equal the oracle's (serialize_packed.rs:375-427 via oracle/capnp_oracle.c)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def _batch(seed, nchunks, p_long, p_adv, p_empty):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(60, 129, nchunks)
    sizes[rng.random(nchunks) < p_empty] = 0
    long_ = rng.random(nchunks) < p_long
    sizes[long_] = rng.integers(129, 700, int(long_.sum()))
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=seed % 3, pz=O.PZ30)
    adv = np.nonzero(rng.random(nchunks) < p_adv)[0]
    for c in adv:  # whole tiles of 8.5-byte words overflow their regions
        t0 = (c // 16) * 16
        a, b = int(offs[t0]), int(offs[min(t0 + 16, nchunks)])
        words[a:b:2] = 0x1112131415161718
        words[a + 1:b:2] = 0x0000212223242526
    return words, offs


def _check(ctx, words, offs, sync, min_provided=0.5):
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    n, total = len(offs) - 1, int(offs[-1])
    out = torch.empty(ctx.batch_bound_bytes(total, n), dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sy = torch.empty(max(ctx.sync_entries(total), 1), dtype=torch.int32, device="cuda")
    ctx.pack_batch_into(dev(words), dev(offs), out, oo, chunks_per_tile=16,
                        sync=sy if sync else None)
    torch.cuda.synchronize()
    got_offs = oo.cpu().numpy().view(np.uint64)
    assert np.array_equal(got_offs, ref_offs), np.nonzero(got_offs != ref_offs)[0][:8]
    got = out[:len(ref)].cpu().numpy()
    if not np.array_equal(got, ref):
        bad = int(np.nonzero(got != ref)[0][0])
        c = int(np.searchsorted(ref_offs, bad, side="right") - 1)
        raise AssertionError(f"bytes differ at {bad} (chunk {c}, tile {c // 16})")
    if sync:
        ref_sync = O.sync_index(ref, ref_offs, offs)
        gs = sy.cpu().numpy().view(np.uint32)[:len(ref_sync)]
        provided = gs != 0xFFFFFFFF
        assert np.array_equal(gs[provided], ref_sync[provided])
        assert provided.mean() > min_provided  # staged tiles provide their entries


@pytest.mark.parametrize("sync", [False, True])
def test_many_tiles_staged(ctx, sync):
    words, offs = _batch(1, 16 * 6000 + 5, 0.0, 0.0, 0.01)
    _check(ctx, words, offs, sync)


@pytest.mark.parametrize("sync", [False, True])
def test_mixed_tile_kinds(ctx, sync):
    words, offs = _batch(2, 16 * 5000 + 11, 0.002, 0.002, 0.02)
    _check(ctx, words, offs, sync)


def test_long_chunks_everywhere(ctx):
    # ~3/4 of the tiles take the streaming size pass (no index entries)
    words, offs = _batch(3, 16 * 2500, 0.08, 0.0, 0.0)
    _check(ctx, words, offs, True, min_provided=0.1)
