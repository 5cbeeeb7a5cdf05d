"""GPU parity of the word-tiled unpack (unpack.hip unpack_wt_kernel): batches
of long chunks decoded through the record sync index in tiles of
capnp_unpack_wt_words() output words that cut chunks anywhere.  The index
comes from the oracle (oracle/packed_oracle.c sync_index over the oracle's
packing), scrambled, or absent; every variant must give the oracle's
statuses, consumed counts and words (the index changes the speed only)."""
import random

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


def _unpack(ctx, packed, in_offs, out_offs, total, sync, utc=0, base=0):
    n = len(in_offs) - 1
    back = torch.zeros(max(total, 1), dtype=torch.int64, device="cuda")
    status = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
    consumed = torch.full((max(n, 1),), -7, dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(packed, dev(in_offs), dev(out_offs), back, status, consumed,
                          chunks_per_tile=utc, sync=sync)
    torch.cuda.synchronize()
    return (back.cpu().numpy().view(np.uint64), status.cpu().numpy()[:n],
            consumed.cpu().numpy().view(np.uint64)[:n])


def _wt_stats(reset=True):
    """(fallback tiles, failed pieces, serially finished chunks) since the
    last reset (capnp_unpack_wt_stats)."""
    import ctypes as C
    from capnp_amd import _lib
    st = (C.c_ulonglong * 4)()
    assert _lib.lib().capnp_unpack_wt_stats(st, int(reset)) == 0
    return tuple(st[:3])


def _index_variants(ref_sync, seed):
    rng = np.random.default_rng(seed)
    bad = ref_sync.copy()
    k = rng.choice(len(bad), max(1, len(bad) // 7))
    bad[k] = rng.integers(0, 1 << 32, len(k), dtype=np.uint64).astype(np.uint32)
    small = ref_sync.copy()  # plausible but wrong: offsets nudged, skips changed
    k = rng.choice(len(small), max(1, len(small) // 11))
    small[k] = (small[k] & 0xFF000000) | ((small[k] & 0xFFFFFF) + rng.integers(1, 40, len(k))
                                          .astype(np.uint32))
    return [("exact", ref_sync), ("scrambled", bad), ("nudged", small),
            ("none", np.full_like(ref_sync, 0xFFFFFFFF))]


def _sizes_long(rng, n):
    # mean well above the word-tile threshold; edges around tile multiples
    tw = 1024
    pool = [tw - 1, tw, tw + 1, 2 * tw - 8, 2 * tw + 8, 3 * tw + 5, 8192, 600, 513, 4097,
            8, 9, 0, 1, 64, 255, 256, 257]
    return [rng.choice(pool) if rng.random() < 0.5 else rng.randrange(1, 9000) for _ in range(n)]


def _check(ctx, words, offs, seed, utcs=(0,)):
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    ref_sync = O.sync_index(ref, ref_offs, offs)
    total = int(offs[-1])
    pk = torch.from_numpy(ref.copy()).cuda()
    for name, sv in _index_variants(ref_sync, seed):
        s = torch.from_numpy(sv.view(np.int32).copy()).cuda()
        for utc in utcs:
            _wt_stats()
            w, st_, used = _unpack(ctx, pk, ref_offs, offs, total, s, utc)
            if name == "exact":  # a valid index keeps every piece on the fast path
                assert _wt_stats() == (0, 0, 0)
            assert (st_ == 0).all(), (name, utc, np.nonzero(st_)[0][:8])
            assert np.array_equal(used, np.diff(ref_offs)), (name, utc)
            bad = np.nonzero(w[:total] != words)[0]
            assert len(bad) == 0, (name, utc, bad[:8])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_word_tiles_round_trip(ctx, kind):
    from capnp_amd import unpack_tile_chunks_for
    rng = random.Random(100 + kind)
    sizes = _sizes_long(rng, 300)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    assert unpack_tile_chunks_for(int(offs[-1]), len(sizes), sync=True) == 0
    words = O.gen_fill(offs, kind0=kind, pz=O.PZ30, id0=kind * 1000)
    _check(ctx, words, offs, kind)


def test_word_tiles_mixed_kinds_and_structures(ctx):
    """Generator kinds mixed per chunk plus hand-made long runs: zero and
    literal runs crossing tile cuts at every phase."""
    rng = random.Random(7)
    chunks = []
    for _ in range(60):
        n = rng.randrange(300, 6000)
        c = np.zeros(n, np.uint64)
        r = rng.random()
        if r < 0.3:  # literal runs with sparse breakers
            c[:] = 0x1112131415161718
            for i in rng.sample(range(n), max(1, n // 700)):
                c[i] = 0x0000000400000001
        elif r < 0.5:  # zero runs with sparse non-zero words
            for i in rng.sample(range(n), max(1, n // 500)):
                c[i] = rng.choice([0x0102030400000000, 0xFFFFFFFFFFFFFFFF, 7])
        else:
            b = c.view(np.uint8)
            b[:] = np.frombuffer(bytes(rng.randrange(256) if rng.random() < 0.5 else 0
                                       for _ in range(8 * n)), np.uint8)
        chunks.append(c)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    _check(ctx, np.concatenate(chunks), offs, 11)


def test_word_tiles_offset_base(ctx):
    """A batch whose words do not start at 0 (a slice of a larger batch):
    tiles follow the global word index of the sync entries."""
    rng = random.Random(5)
    sizes = _sizes_long(rng, 80)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30, id0=3)
    st, ref, ref_offs = O.pack_batch(words, offs)
    ref_sync = O.sync_index(ref, ref_offs, offs)
    k = 3
    pk = torch.from_numpy(ref.copy()).cuda()
    s = torch.from_numpy(ref_sync.view(np.int32).copy()).cuda()
    total = int(offs[-1])
    w, st_, used = _unpack(ctx, pk, ref_offs[k:], offs[k:], total, s)
    assert (st_ == 0).all()
    assert np.array_equal(used, np.diff(ref_offs[k:]))
    a = int(offs[k])
    assert np.array_equal(w[a:total], words[a:])


def test_word_tiles_errors_vs_oracle(ctx):
    """Long chunks truncated, corrupted, mis-sized or with trailing bytes;
    the index is the encoder's (from the uncorrupted packing), scrambled or
    absent: statuses, consumed counts and the words of good chunks equal the
    oracle's."""
    rng = random.Random(31)
    packed_chunks, lens, orig, orig_lens = [], [], [], []
    for i in range(160):
        n = rng.choice([600, 1024, 1500, 2048, 3000, 5000, 8192, 12])
        w = O.gen_fill(np.array([0, n], np.uint64), kind0=rng.randrange(3), pz=O.PZ30, id0=i)
        st, k = O.pack(w.tobytes())
        orig.append(k)
        orig_lens.append(n)
        k = bytearray(k)
        r = rng.random()
        if r < 0.15 and len(k) > 1:
            k = k[:rng.randrange(len(k))]
        elif r < 0.35 and len(k):
            for _ in range(rng.randrange(1, 3)):
                k[rng.randrange(len(k))] = rng.choice([0, 0xFF, rng.randrange(256)])
        elif r < 0.45:
            n = max(0, n + rng.choice([-9, -1, 1, 8]))
        elif r < 0.55:
            k = k + bytes([rng.randrange(256) for _ in range(rng.randrange(1, 12))])
        packed_chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in packed_chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(packed_chunks), np.uint8)
    ref_words, ref_st, ref_used = O.unpack_batch(packed, in_offs, out_offs)
    assert (ref_st != 0).sum() > 20 and (ref_st == 0).sum() > 60
    total = int(out_offs[-1])
    # the encoder's index: from the clean packing and the original lengths
    # (after a mis-sized chunk it describes shifted words: wrong, as it may be)
    o_in = np.concatenate([[0], np.cumsum([len(k) for k in orig])]).astype(np.uint64)
    o_out = np.concatenate([[0], np.cumsum(orig_lens)]).astype(np.uint64)
    enc = O.sync_index(np.frombuffer(b"".join(orig), np.uint8), o_in, o_out)
    ne = -(-total // O.sync_words())
    enc = np.concatenate([enc, np.full(max(0, ne - len(enc)), 0xFFFFFFFF, np.uint32)])[:ne]
    pk = torch.from_numpy(packed.copy()).cuda()
    ok = ref_st == 0
    for name, sv in _index_variants(enc, 3)[:2] + [("none", np.full(ne, 0xFFFFFFFF, np.uint32))]:
        s = torch.from_numpy(sv.view(np.int32).copy()).cuda()
        gw, g_st, g_used = _unpack(ctx, pk, in_offs, out_offs, total, s)
        assert np.array_equal(g_st, ref_st), (name, np.nonzero(g_st != ref_st)[0][:8])
        assert np.array_equal(g_used, ref_used), name
        for c in np.nonzero(ok)[0]:
            a, b = int(out_offs[c]), int(out_offs[c + 1])
            assert np.array_equal(gw[a:b], ref_words[a:b]), (name, c)


# --------------------------------------------------------------- word-tile pack
def _check_pack(ctx, words, offs, base=0):
    """Pack in word tiles (chunks_per_tile 0, mean >= WORD_TILE_MEAN): bytes,
    offsets and the whole sync index equal the oracle's; then the word-tile
    unpack through the GPU's own index returns the words."""
    from capnp_amd import tile_chunks_for
    n, total = len(offs) - 1, int(offs[-1])
    assert tile_chunks_for(total - int(offs[0]), n) == 0
    st, ref, ref_offs = O.pack_batch(words[int(offs[0]):], offs - offs[0])
    assert st == 0
    ref_sync = O.sync_index(ref, ref_offs, offs - offs[0]) if offs[0] == 0 else None
    dw = torch.from_numpy(np.ascontiguousarray(words).view(np.int64)).cuda()
    do = dev(offs)
    cap = ctx.batch_bound_bytes(total, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sync = torch.full((max(ctx.sync_entries(total), 1),), -5, dtype=torch.int32, device="cuda")
    ctx.pack_batch_into(dw, do, out, oo, chunks_per_tile=0, sync=sync)
    torch.cuda.synchronize()
    go = oo.cpu().numpy().view(np.uint64)
    assert np.array_equal(go - go[0], ref_offs), np.nonzero(go - go[0] != ref_offs)[0][:8]
    got = out[int(go[0]):int(go[-1])].cpu().numpy()
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]
    gs = sync.cpu().numpy().view(np.uint32)
    if ref_sync is not None:
        bad = np.nonzero(gs[:len(ref_sync)] != ref_sync)[0]
        assert len(bad) == 0, (bad[:8], gs[bad[:4]], ref_sync[bad[:4]])
    back = torch.zeros(max(total, 1), dtype=torch.int64, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    consumed = torch.empty(n, dtype=torch.int64, device="cuda")
    _wt_stats()
    ctx.unpack_batch_into(out, oo, do, back, status, consumed, chunks_per_tile=0, sync=sync)
    torch.cuda.synchronize()
    assert _wt_stats() == (0, 0, 0)
    assert int((status != 0).sum()) == 0
    assert np.array_equal(consumed.cpu().numpy().view(np.uint64), np.diff(go))
    b = back.cpu().numpy().view(np.uint64)
    assert np.array_equal(b[int(offs[0]):total], words[int(offs[0]):total])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_word_tile_pack(ctx, kind):
    rng = random.Random(200 + kind)
    sizes = _sizes_long(rng, 300)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=kind, pz=O.PZ30, id0=kind * 77)
    _check_pack(ctx, words, offs)


def test_word_tile_pack_structures(ctx):
    """Runs of every length and phase across range (512-word) and tile
    (2048-word) cuts: all-zero and all-0xFF stretches far longer than 255
    words (heads every 256 from the last sure head), literal runs of words
    with one zero byte, sparse breakers, empty and one-word chunks."""
    rng = random.Random(9)
    chunks = []
    for i in range(80):
        n = rng.choice([0, 1, 7, 600, 1500, 2048, 2049, 4096, 5000, 9000])
        c = np.zeros(n, np.uint64)
        r = i % 5
        if r == 0:  # all 0xFF tags, sparse breakers
            c[:] = 0x1112131415161718
            for j in rng.sample(range(n), min(n, rng.randrange(0, 4))):
                c[j] = 0x0000000400000001
        elif r == 1:  # zeros with sparse literal words
            for j in rng.sample(range(n), min(n, rng.randrange(0, 4))):
                c[j] = 0xFFFFFFFFFFFFFFFF
        elif r == 2:  # words with exactly one zero byte, some full
            b = c.view(np.uint8).reshape(-1, 8) if n else None
            for j in range(n):
                v = [rng.randrange(1, 256) for _ in range(8)]
                if rng.random() < 0.7:
                    v[rng.randrange(8)] = 0
                b[j] = v
        elif r == 3:  # mixed random
            b = c.view(np.uint8)
            b[:] = np.frombuffer(bytes(rng.randrange(256) if rng.random() < 0.4 else 0
                                       for _ in range(8 * n)), np.uint8)
        else:  # long literal run then long zero run
            c[:n // 2] = 0x0101010101010101
        chunks.append(c)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    _check_pack(ctx, np.concatenate(chunks), offs)


def test_word_tile_pack_deep_stretches(ctx):
    """Stretches of tens of thousands of all-zero or all-0xFF words (plan
    entries deferred and taken from the range 512 words back), entered at
    every phase after a random prefix, with a lone 7-byte word or a breaker
    deep inside some of them, and runs of 7-byte words (no closed form)."""
    rng = random.Random(41)
    chunks = []
    for i in range(24):
        pre = rng.randrange(0, 700)
        n = rng.choice([3000, 9000, 20000, 41000])
        c = np.zeros(pre + n, np.uint64)
        b = c.view(np.uint8).reshape(-1, 8)
        b[:pre] = np.frombuffer(bytes(rng.randrange(256) if rng.random() < 0.5 else 0
                                      for _ in range(8 * pre)), np.uint8).reshape(-1, 8)
        kind = i % 4
        if kind == 1:
            c[pre:] = 0x1112131415161718
        elif kind == 2:
            c[pre:] = 0x1112131400161718  # 7-byte words: literal runs, no closed form
        elif kind == 3:
            c[pre:] = 0x2122232425262728
            c[pre + rng.randrange(n)] = 0x2122232425002728
        if i % 3 == 0:
            c[pre + rng.randrange(n)] = 0x0000000400000001
        chunks.append(c)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    _check_pack(ctx, np.concatenate(chunks), offs)


def test_word_tile_pack_offset_base(ctx):
    rng = random.Random(12)
    sizes = _sizes_long(rng, 60)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30, id0=5)
    k = 5
    _check_pack(ctx, words, offs[k:])
