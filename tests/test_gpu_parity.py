"""GPU parity: the gfx950 kernels against the CPU oracle, bit for bit.

Every test goes through the C ABI (libcapnp_packed.so).  Small cases are
compared byte-for-byte with the oracle (and its golden vectors); the full
BASELINE sizes are checked through size-independent properties (round trip,
offsets = sizes, sampled chunk bytes against the oracle)."""
import json
import os
import random

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_packing.json")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def dev(a, dtype=torch.int64):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64 if dtype == torch.int64 else
                                                         np.uint8)).cuda()


# ---------------------------------------------------------------- host API
def test_golden_pack_unpack(ctx, golden):
    from capnp_amd import serialize_packed as sp
    from capnp_amd import _lib
    import ctypes as C
    L = _lib.lib()
    for v in golden["packing"]:
        u, k = bytes(v["unpacked"]), bytes(v["packed"])
        out = bytearray()
        sp.PackedWrite(out, ctx).write_all(u)
        assert bytes(out) == k, v
        r = sp.PackedRead(sp.SliceRead(k), ctx)
        assert r.read_exact(len(u)) == u
        assert r.inner.is_empty()


def test_golden_unpack_errors(ctx, golden):
    from capnp_amd import serialize_packed as sp, CapnpError
    names = {2: "PrematureEndOfPackedInput", 3: "PackedInputDidNotEndCleanlyOnASegmentBoundary",
             4: "FailedToFillTheWholeBuffer"}
    for v in golden["unpack_errors"]:
        with pytest.raises(CapnpError) as e:
            sp.PackedRead(sp.SliceRead(bytes(v["packed"])), ctx).read_exact(v["out_len"])
        assert e.value.status == O.STATUS[v["status"]], (v, e.value)
    for v in golden["unpacks_to"]:
        r = sp.PackedRead(sp.SliceRead(bytes(v["packed"])), ctx)
        assert r.read_exact(len(v["unpacked"])) == bytes(v["unpacked"])


def test_golden_read_message(ctx, golden):
    from capnp_amd import serialize_packed as sp, CapnpError
    m = sp.read_message(bytes([0x11, 4, 1, 0, 1, 0, 0]), ctx=ctx)
    assert [len(s) for s in m.segments()] == [1, 0, 0, 0, 0]
    assert sp.try_read_message(b"", ctx=ctx) is None
    with pytest.raises(CapnpError) as e:
        sp.read_message(b"", ctx=ctx)
    assert e.value.kind == "PrematureEndOfFile"
    # no-alloc path reads the table rest 8 bytes at a time
    with pytest.raises(CapnpError) as e:
        sp.read_message_no_alloc(bytes([0x11, 4, 1, 0, 1, 0, 0]), np.zeros(64, np.uint64), ctx=ctx)
    assert e.value.kind == "PackedInputDidNotEndCleanlyOnASegmentBoundary"


def _rand_segment(rng, n):
    kind = rng.random()
    w = np.zeros(n, np.uint64)
    b = w.view(np.uint8)
    for i in range(n):
        r = rng.random()
        if kind < 0.25:  # zero heavy
            if r < 0.1:
                b[8 * i:8 * i + 8] = [rng.randrange(256) for _ in range(8)]
        elif kind < 0.5:  # literal heavy
            vals = [rng.randrange(1, 256) for _ in range(8)]
            if r < 0.05:
                vals[rng.randrange(8)] = 0
                vals[rng.randrange(8)] = 0
            elif r < 0.3:
                vals[rng.randrange(8)] = 0
            b[8 * i:8 * i + 8] = vals
        else:
            if r < 0.3:
                continue
            b[8 * i:8 * i + 8] = [rng.randrange(256) if rng.random() < 0.56 else 0
                                  for _ in range(8)]
    return w


def test_message_round_trip_vs_oracle(ctx):
    from capnp_amd import serialize_packed as sp
    rng = random.Random(11)
    for _ in range(60):
        segs = [_rand_segment(rng, rng.choice([0, 1, 3, 64, 65, 200, 300]))
                for _ in range(rng.randrange(1, 7))]
        out = bytearray()
        sp.write_message(out, segs, ctx=ctx)
        st, ref = O.write_message(segs)
        assert st == 0 and bytes(out) == ref
        r = sp.SliceRead(bytes(out) + b"\x00\x00")  # trailing bytes stay unconsumed
        m = sp.read_message(r, ctx=ctx)
        assert r.pos == len(out)
        for a, b in zip(segs, m.segments()):
            assert np.array_equal(a, b)
        buf = np.zeros(8192, np.uint64)
        if len(segs) >= 3 and all(len(s) == 0 for s in segs[1:]):
            continue
        m2 = sp.read_message_no_alloc(bytes(out), buf, ctx=ctx)
        for a, b in zip(segs, m2.segments()):
            assert np.array_equal(a, b)


def _runs_segment(rng, n):
    """Words built from runs whose lengths straddle the split ranges of a
    long last segment (msg_pack_kernel: 64-word multiples per wave): zero
    runs and 0xFF runs of 1..700 words (past the 255-word cap), runs of
    words with one zero byte (absorbed by a 0xFF run, not heads of one),
    and breakers."""
    w = np.zeros(n, np.uint64)
    i = 0
    while i < n:
        k = min(n - i, rng.choice([1, 2, 63, 64, 65, 127, 128, 129, 191, 255, 256, 257, 300,
                                   511, 700]))
        kind = rng.randrange(5)
        if kind == 0:
            pass  # zero words
        elif kind == 1:
            w[i:i + k] = 0x0102030405060708  # 0xFF words
        elif kind == 2:
            w[i] = 0x1111111111111111
            w[i + 1:i + k] = 0x0011223344556677  # one zero byte: absorbed by a 0xFF run
        elif kind == 3:
            w[i:i + k] = 0x0000FF000000AB00  # 2 non-zero bytes: breakers
        else:
            for j in range(i, i + k):
                w[j] = rng.getrandbits(64) & rng.choice([0, 0xFFFFFFFFFFFFFFFF,
                                                          0x00FF00FF00FF00FF])
        i += k
    return w


@pytest.mark.parametrize("seed", range(6))
def test_message_split_segment_vs_oracle(ctx, seed):
    """A long last segment is packed by all four waves of the one-launch
    write (csrc/pack.hip msg_pack_kernel, ranges with the run state carried
    in and the open run's count continued past the range end): byte-equal
    to the oracle's write_message for segments of 256..8184 words built from
    runs across the range boundaries, after 0..3 short segments."""
    from capnp_amd import serialize_packed as sp
    rng = random.Random(1000 + seed)
    for n in (256, 257, 300, 511, 1024, 1500, 2047, 4000, 4096 - 8, 6000, 8192 - 8):
        head = [_rand_segment(rng, rng.choice([0, 1, 5])) for _ in range(rng.randrange(0, 4))]
        segs = head + [_runs_segment(rng, n)]
        out = bytearray()
        sp.write_message(out, segs, ctx=ctx)
        st, ref = O.write_message(segs)
        assert st == 0 and bytes(out) == ref, (seed, n)


# ---------------------------------------------------------------- batch API
def _check_batch(ctx, words, offs, tc=0, utcs=(0, 1, 7, 256)):
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    dw, do = dev(words), dev(offs)
    packed, poffs = ctx.pack_batch(dw, do, chunks_per_tile=tc)
    torch.cuda.synchronize()
    got = packed.cpu().numpy()
    goffs = poffs.cpu().numpy().view(np.uint64)
    assert np.array_equal(goffs, ref_offs), "offsets differ"
    if not np.array_equal(got, ref):
        bad = np.nonzero(got != ref)[0][0]
        c = int(np.searchsorted(ref_offs, bad, side="right") - 1)
        raise AssertionError(f"packed bytes differ at {bad} (chunk {c}, words "
                             f"{offs[c + 1] - offs[c]})")
    # unpack tile sizes: staged (LDS) path, tiny tiles, and tiles that overflow
    # the LDS tables (global path)
    for utc in utcs:
        back, status, consumed = ctx.unpack_batch(packed, poffs, do, chunks_per_tile=utc)
        torch.cuda.synchronize()
        assert (status.cpu().numpy() == 0).all(), utc
        assert np.array_equal(consumed.cpu().numpy().view(np.uint64), np.diff(ref_offs)), utc
        assert np.array_equal(back.cpu().numpy().view(np.uint64), words), utc


@pytest.mark.parametrize("tc", [0, 1, 3, 16, 64])
def test_batch_edge_sizes(ctx, tc):
    sizes = [0, 1, 2, 7, 8, 63, 64, 65, 127, 128, 129, 191, 192, 255, 256, 257, 320, 511, 512,
             513, 1000, 0, 0, 5]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for kind in (0, 1, 2):
        words = O.gen_fill(offs, kind0=kind, pz=O.PZ30)
        _check_batch(ctx, words, offs, tc)


def test_batch_random_structures(ctx):
    rng = random.Random(5)
    segs = [_rand_segment(rng, rng.choice([0, 1, 5, 64, 100, 128, 256, 300, 700]))
            for _ in range(120)]
    offs = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.uint64)
    words = np.concatenate(segs)
    _check_batch(ctx, words, offs)
    _check_batch(ctx, words, offs, tc=1)


def test_batch_long_runs(ctx):
    # zero and literal runs longer than 255 words, every alignment vs 64
    chunks = []
    for n in (255, 256, 257, 300, 511, 512, 513, 1023, 1500):
        for lead in (0, 1, 63):
            z = np.zeros(n + lead, np.uint64)
            z[:lead] = 0x0102030400000000
            chunks.append(z)
            lit = np.full(n + lead, 0x1112131415161718, np.uint64)
            lit[:lead] = 0x0000000400000001
            chunks.append(lit)
            mix = np.full(n + lead, 0x11121314151617, np.uint64)  # one zero byte
            mix[lead] = 0x1112131415161718
            chunks.append(mix)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    _check_batch(ctx, np.concatenate(chunks), offs)


def test_batch_misaligned_output(ctx):
    sizes = np.random.default_rng(3).integers(0, 200, 300)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    st, ref, ref_offs = O.pack_batch(words, offs)
    dw, do = dev(words), dev(offs)
    n = len(sizes)
    cap = len(ref) + 64
    for mis in (1, 3, 8, 15):
        buf = torch.full((cap + 32,), 0xEE, dtype=torch.uint8, device="cuda")
        out = buf[mis:mis + cap]
        oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        ctx.pack_batch_into(dw, do, out, oo)
        torch.cuda.synchronize()
        b = buf.cpu().numpy()
        assert (b[:mis] == 0xEE).all()
        assert np.array_equal(b[mis:mis + len(ref)], ref)
        assert (b[mis + len(ref):mis + len(ref) + 8] == 0xEE).all()


def test_batch_small_capacity_writes_nothing_past_cap(ctx):
    offs = np.arange(0, 129 * 64, 128, dtype=np.uint64)[:65]
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    st, ref, ref_offs = O.pack_batch(words, offs)
    cap = len(ref) // 2
    buf = torch.full((len(ref) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    oo = torch.empty(65, dtype=torch.int64, device="cuda")
    ctx.pack_batch_into(dev(words), dev(offs), buf[:cap], oo)
    torch.cuda.synchronize()
    assert int(oo[-1]) == len(ref)
    assert (buf[cap:].cpu().numpy() == 0xEE).all()


def test_unpack_error_statuses_vs_oracle(ctx):
    rng = random.Random(17)
    packed_chunks, lens = [], []
    for _ in range(600):
        n = rng.choice([1, 2, 5, 40, 64, 65, 130])
        w = _rand_segment(rng, n)
        st, k = O.pack(w.tobytes())
        k = bytearray(k)
        r = rng.random()
        if r < 0.3 and len(k) > 1:
            k = k[:rng.randrange(len(k))]          # truncate
        elif r < 0.5 and len(k):
            k[rng.randrange(len(k))] = rng.choice([0, 0xFF, rng.randrange(256)])  # corrupt
        elif r < 0.6:
            n = max(0, n + rng.choice([-3, -1, 1, 4]))  # wrong output size
        packed_chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in packed_chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(packed_chunks), np.uint8)
    ref_words, ref_st, ref_used = O.unpack_batch(packed, in_offs, out_offs)
    pk = torch.from_numpy(packed.copy()).cuda() if len(packed) else torch.zeros(1, dtype=torch.uint8, device="cuda")
    ok = ref_st == 0
    assert ok.sum() > 100 and (~ok).sum() > 100
    for utc in (0, 1, 13, 64, 256):
        words, status, consumed = ctx.unpack_batch(pk, dev(in_offs), dev(out_offs),
                                                   chunks_per_tile=utc)
        torch.cuda.synchronize()
        g_st = status.cpu().numpy()
        assert np.array_equal(g_st, ref_st), (utc, np.nonzero(g_st != ref_st))
        assert np.array_equal(consumed.cpu().numpy().view(np.uint64), ref_used), utc  # error chunks too
        gw = words.cpu().numpy().view(np.uint64)
        for c in np.nonzero(ok)[0]:
            a, b = int(out_offs[c]), int(out_offs[c + 1])
            assert np.array_equal(gw[a:b], ref_words[a:b]), (utc, c)


def test_generator_matches_oracle(ctx):
    from capnp_amd import _lib
    sizes = np.random.default_rng(0).integers(0, 400, 500)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    kinds = np.random.default_rng(1).integers(0, 3, 500).astype(np.uint8)
    for pz in (O.PZ30, O.PZ80):
        ref = O.gen_fill(offs, kinds=kinds, pz=pz, id0=77)
        w = torch.empty(int(offs[-1]), dtype=torch.int64, device="cuda")
        ctx.gen_batch(w, dev(offs), pz_thresh=pz,
                      kinds=torch.from_numpy(kinds).cuda(), id0=77)
        torch.cuda.synchronize()
        assert np.array_equal(w.cpu().numpy().view(np.uint64), ref)


@pytest.mark.parametrize("pz", [O.PZ30, O.PZ80])
def test_full_size_config_round_trip(ctx, pz):
    """BASELINE configs 2/3 shape (1 Mi x 1 KiB): round trip on the device,
    offsets = chunk sizes, and 2048 sampled chunks byte-equal to the oracle."""
    n, cw = 1 << 20, 128
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=pz)
    packed, poffs = ctx.pack_batch(words, offs)
    back, status, consumed = ctx.unpack_batch(packed, poffs, offs)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(back, words)
    assert torch.equal(consumed, poffs[1:] - poffs[:-1])
    idx = np.random.default_rng(9).choice(n, 2048, replace=False)
    po = poffs.cpu().numpy()
    pk = packed.cpu().numpy()
    for c in idx[:2048]:
        w = O.gen_fill(np.array([0, cw], np.uint64), pz=pz, id0=int(c))
        st, k = O.pack(w.tobytes())
        assert pk[po[c]:po[c + 1]].tobytes() == k


def _check_sampled(packed, poffs, ids_kinds, pz, cw_of):
    po = poffs.cpu().numpy()
    for c, kind in ids_kinds:
        w = O.gen_fill(np.array([0, cw_of(c)], np.uint64), kinds=np.array([kind], np.uint8),
                       pz=pz, id0=int(c))
        st, k = O.pack(w.tobytes())
        got = packed[int(po[c]):int(po[c + 1])].cpu().numpy().tobytes()
        assert got == k, f"chunk {c} (kind {kind}, {cw_of(c)} words) differs"


def test_config3_high_sparsity_4gib_packed(ctx):
    """BASELINE config 3: >= 80 % zero words, 4 GiB of packed input
    (~23.4 Mi chunks x 1 KiB, ~22 GiB unpacked): device round trip, status,
    consumed bytes, and 512 sampled chunks byte-equal to the oracle."""
    from capnp_amd import unpack_tile_chunks_for
    cw = 128
    n = 23_400_000
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=O.PZ80)
    packed, poffs = ctx.pack_batch(words, offs)
    assert packed.numel() >= 4 * 10**9 * 0.93
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    consumed = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed,
                          chunks_per_tile=unpack_tile_chunks_for(n * cw, n))
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(back, words)
    assert torch.equal(consumed, poffs[1:] - poffs[:-1])
    del back, words
    idx = np.random.default_rng(3).choice(n, 512, replace=False)
    _check_sampled(packed, poffs, [(int(c), 0) for c in idx], O.PZ80, lambda c: cw)


def test_config4_mixed_sizes_round_trip(ctx):
    """BASELINE config 4: chunk sizes log-uniform in [8, 8192] words (64 B -
    64 KiB), ~1 GiB, 80 % config-2 words / 10 % long zero runs / 10 % long
    literal runs: round trip and sampled chunks (the largest included)
    byte-equal to the oracle."""
    from capnp_amd import tile_chunks_for, unpack_tile_chunks_for
    rng = np.random.default_rng(4)
    target = (1 << 30) // 8
    sizes = []
    total = 0
    while total < target:
        s = int(np.exp(rng.uniform(np.log(8), np.log(8193))))
        sizes.append(s)
        total += s
    n = len(sizes)
    kinds = rng.choice(3, size=n, p=[0.8, 0.1, 0.1]).astype(np.uint8)
    offs_h = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    offs = dev(offs_h)
    words = torch.empty(total, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=O.PZ30, kinds=torch.from_numpy(kinds).cuda())
    packed, poffs = ctx.pack_batch(words, offs, chunks_per_tile=tile_chunks_for(total, n))
    back, status, consumed = ctx.unpack_batch(packed, poffs, offs,
                                              chunks_per_tile=unpack_tile_chunks_for(total, n))
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(back, words)
    assert torch.equal(consumed, poffs[1:] - poffs[:-1])
    big = np.argsort(sizes)[-32:]
    idx = np.concatenate([big, rng.choice(n, 224, replace=False)])
    _check_sampled(packed, poffs, [(int(c), int(kinds[c])) for c in idx], O.PZ30,
                   lambda c: sizes[c])


def test_config5_full_shard_round_trip(ctx):
    """BASELINE config 5's per-GPU shard: 8 Mi x 1 KiB = 8 GiB of words (the
    64 GiB batch over 8 GPUs, bench.py --workload config5), packed with the
    record sync index and unpacked through it on one GPU: exact round trip,
    statuses, consumed bytes, and 256 sampled chunks byte-equal to the
    oracle (shard 0: generator ids from 0, as rank 0 of the bench)."""
    from capnp_amd import tile_chunks_for, unpack_tile_chunks_for
    n, cw = 8 << 20, 128
    total = n * cw
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(total, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=O.PZ30, id0=0)
    cap = ctx.batch_bound_bytes(total, n)
    packed = torch.empty(cap, dtype=torch.uint8, device="cuda")
    poffs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sync = torch.empty(ctx.sync_entries(total), dtype=torch.int32, device="cuda")
    ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tile_chunks_for(total, n),
                        sync=sync)
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    consumed = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed,
                          chunks_per_tile=unpack_tile_chunks_for(total, n, sync=True), sync=sync)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(back, words)
    assert torch.equal(consumed, poffs[1:] - poffs[:-1])
    del back
    idx = np.random.default_rng(55).choice(n, 256, replace=False)
    _check_sampled(packed, poffs, [(int(c), 0) for c in idx], O.PZ30, lambda c: cw)


# ------------------------------------------------------- record sync index
def _pack_sync(ctx, dw, do, n, total, tc=0):
    cap = ctx.batch_bound_bytes(total, n)
    out = torch.empty(max(cap, 1), dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sync = torch.empty(max(ctx.sync_entries(total), 1), dtype=torch.int32, device="cuda")
    ctx.pack_batch_into(dw, do, out, oo, chunks_per_tile=tc, sync=sync)
    return out, oo, sync


def _unpack_sync(ctx, packed, poffs, do, total, n, sync, utc=0):
    back = torch.empty(max(total, 1), dtype=torch.int64, device="cuda")
    status = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    consumed = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(packed, poffs, do, back, status, consumed, chunks_per_tile=utc,
                          sync=sync)
    torch.cuda.synchronize()
    return (back.cpu().numpy().view(np.uint64)[:total], status.cpu().numpy()[:n],
            consumed.cpu().numpy().view(np.uint64)[:n])


def _check_sync_batch(ctx, words, offs, tc=0, utcs=(0, 1, 7, 64)):
    """Pack with the record sync index (bytes == oracle, index == oracle
    where provided) and unpack through it (== the words, status OK); then
    the same unpack with a scrambled index and with no entries: the result
    must not change (segments that do not meet fall back to the serial walk)."""
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    n, total = len(offs) - 1, int(offs[-1])
    ref_sync = O.sync_index(ref, ref_offs, offs)
    dw, do = dev(words), dev(offs)
    out, oo, sync = _pack_sync(ctx, dw, do, n, total, tc)
    torch.cuda.synchronize()
    assert np.array_equal(oo.cpu().numpy().view(np.uint64), ref_offs)
    assert np.array_equal(out[:len(ref)].cpu().numpy(), ref)
    gs = sync.cpu().numpy().view(np.uint32)[:len(ref_sync)]
    provided = gs != 0xFFFFFFFF
    assert np.array_equal(gs[provided], ref_sync[provided]), np.nonzero(gs != ref_sync)
    packed = out[:max(len(ref), 1)]
    rng = np.random.default_rng(total)
    bad = ref_sync.copy()
    if len(bad):
        k = rng.choice(len(bad), max(1, len(bad) // 5))
        bad[k] = rng.integers(0, 1 << 32, len(k), dtype=np.uint64).astype(np.uint32)
    variants = [sync, torch.from_numpy(bad.view(np.int32).copy()).cuda() if len(bad) else sync,
                torch.full_like(sync, -1)]
    for utc in utcs:
        for sv in variants:
            w, s, c = _unpack_sync(ctx, packed, oo, do, total, n, sv, utc)
            assert (s == 0).all(), utc
            assert np.array_equal(c, np.diff(ref_offs)), utc
            assert np.array_equal(w, words), utc


@pytest.mark.parametrize("tc", [0, 1, 3, 16])
def test_sync_edge_sizes(ctx, tc):
    sizes = [0, 1, 2, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257, 320, 511,
             512, 513, 1000, 0, 0, 5]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for kind in (0, 1, 2):
        words = O.gen_fill(offs, kind0=kind, pz=O.PZ30)
        _check_sync_batch(ctx, words, offs, tc)


def test_sync_random_structures(ctx):
    rng = random.Random(23)
    segs = [_rand_segment(rng, rng.choice([0, 1, 5, 31, 33, 64, 100, 128, 256, 300]))
            for _ in range(200)]
    offs = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.uint64)
    _check_sync_batch(ctx, np.concatenate(segs), offs)


def test_sync_long_runs(ctx):
    chunks = []
    for n in (31, 32, 33, 255, 256, 257, 300, 500):
        for lead in (0, 1, 31, 63):
            z = np.zeros(n + lead, np.uint64)
            z[:lead] = 0x0102030400000000
            chunks.append(z)
            lit = np.full(n + lead, 0x1112131415161718, np.uint64)
            lit[:lead] = 0x0000000400000001
            chunks.append(lit)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    _check_sync_batch(ctx, np.concatenate(chunks), offs, utcs=(0, 3))


def test_pack_region_overflow(ctx):
    """Adversarial ranges (a 0xFF word then a 6-byte word, 8.5 packed bytes
    per word) overflow the staged regions: those tiles take the streaming
    path (bytes and offsets exact, no index entries); mixed with tiles that
    fit and with empty and short chunks."""
    rng = random.Random(61)
    chunks = []
    for i in range(300):
        n = rng.choice([0, 1, 64, 128, 128, 128, 200, 256])
        c = np.zeros(n, np.uint64)
        if i % 3:
            c[0::2] = 0x1112131415161718
            c[1::2] = 0x0000212223242526
        else:
            b = c.view(np.uint8)
            b[:] = np.frombuffer(bytes(rng.randrange(256) if rng.random() < 0.6 else 0
                                       for _ in range(8 * n)), np.uint8)
        chunks.append(c)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    words = np.concatenate(chunks)
    for tc in (0, 4, 16):
        _check_sync_batch(ctx, words, offs, tc, utcs=(0, 7))
    st, ref, ref_offs = O.pack_batch(words, offs)
    out = torch.zeros(ctx.batch_bound_bytes(int(offs[-1]), len(offs) - 1), dtype=torch.uint8,
                      device="cuda")
    oo = torch.empty(len(offs), dtype=torch.int64, device="cuda")
    ctx.pack_batch_into(dev(words), dev(offs), out, oo)
    torch.cuda.synchronize()
    assert np.array_equal(oo.cpu().numpy().view(np.uint64), ref_offs)
    assert np.array_equal(out[:len(ref)].cpu().numpy(), ref)


def test_sync_unpack_error_statuses_vs_oracle(ctx):
    """Malformed chunks through the sync path (index garbage or absent):
    statuses, consumed counts and the words of good chunks equal the oracle."""
    rng = random.Random(29)
    packed_chunks, lens = [], []
    for _ in range(600):
        n = rng.choice([1, 2, 5, 31, 32, 40, 64, 65, 130])
        w = _rand_segment(rng, n)
        st, k = O.pack(w.tobytes())
        k = bytearray(k)
        r = rng.random()
        if r < 0.3 and len(k) > 1:
            k = k[:rng.randrange(len(k))]
        elif r < 0.5 and len(k):
            k[rng.randrange(len(k))] = rng.choice([0, 0xFF, rng.randrange(256)])
        elif r < 0.6:
            n = max(0, n + rng.choice([-3, -1, 1, 4]))
        elif r < 0.7:
            k = k + bytes([rng.randrange(256) for _ in range(rng.randrange(1, 12))])
        packed_chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in packed_chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(packed_chunks), np.uint8)
    ref_words, ref_st, ref_used = O.unpack_batch(packed, in_offs, out_offs)
    total, n = int(out_offs[-1]), len(lens)
    pk = torch.from_numpy(packed.copy()).cuda()
    ok = ref_st == 0
    ne = -(-total // O.sync_words())
    garbage = torch.from_numpy(np.random.default_rng(2).integers(
        0, 1 << 32, ne, dtype=np.uint64).astype(np.uint32).view(np.int32)).cuda()
    small = torch.from_numpy(np.random.default_rng(3).integers(
        0, 1 << 12, ne, dtype=np.uint64).astype(np.uint32).view(np.int32)).cuda()
    for sv in (garbage, small, torch.full((ne,), -1, dtype=torch.int32, device="cuda")):
        for utc in (0, 1, 13):
            gw, g_st, g_used = _unpack_sync(ctx, pk, dev(in_offs), dev(out_offs), total, n, sv,
                                            utc)
            assert np.array_equal(g_st, ref_st), (utc, np.nonzero(g_st != ref_st))
            assert np.array_equal(g_used, ref_used), utc  # error chunks too
            for c in np.nonzero(ok)[0]:
                a, b = int(out_offs[c]), int(out_offs[c + 1])
                assert np.array_equal(gw[a:b], ref_words[a:b]), (utc, c)


@pytest.mark.parametrize("pz", [O.PZ30, O.PZ80])
def test_sync_full_size_config(ctx, pz):
    """Config 2/3 shape (1 Mi x 1 KiB) through the sync path: index == the
    oracle's on sampled tiles, device round trip exact."""
    n, cw = 1 << 20, 128
    total = n * cw
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(total, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=pz)
    out, oo, sync = _pack_sync(ctx, words, offs, n, total)
    torch.cuda.synchronize()
    gs = sync.cpu().numpy().view(np.uint32)
    assert (gs != 0xFFFFFFFF).all()
    w, s, c = _unpack_sync(ctx, out, oo, offs, total, n, sync)
    assert (s == 0).all()
    assert np.array_equal(w, words.cpu().numpy().view(np.uint64))
    po = oo.cpu().numpy().view(np.uint64)
    assert np.array_equal(c, np.diff(po))
    pk = out.cpu().numpy()
    for ch in np.random.default_rng(5).choice(n, 256, replace=False):
        a, b = int(po[ch]), int(po[ch + 1])
        ref = O.sync_index(pk[a:b], np.array([0, b - a], np.uint64),
                           np.array([0, cw], np.uint64))
        k = cw // O.sync_words()
        assert np.array_equal(gs[ch * k:ch * k + k], ref), ch
