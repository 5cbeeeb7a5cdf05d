"""Message-boundary discovery in a concatenated packed stream with no byte
index (capnp_gpu_find_messages + capnp_gpu_read_messages)
against the oracle's try_read_message loop (serialize.rs:310-325,
serialize_packed.rs:246-255): per message segments and consumed bytes, and
how the loop ends (None after a clean end, else the failing status), on
valid, truncated, garbage-tailed and over-limit streams."""
import random

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


def _segments(rng, big=False):
    segs = []
    for _ in range(rng.choice([1, 1, 1, 2, 3, 4, 7, 30])):
        n = rng.choice([0, 1, 5, 16, 100, 600] + ([3000, 20000] if big else []))
        kind = rng.random()
        if kind < 0.1:  # long literal stretches
            ws = [rng.getrandbits(64) | 0x0101010101010101 for _ in range(n)]
        elif kind < 0.2:  # mostly zeros
            ws = [rng.getrandbits(64) if rng.random() < 0.02 else 0 for _ in range(n)]
        else:
            ws = []
            for _ in range(n):
                b = [rng.getrandbits(8) if rng.random() < 0.56 else 0 for _ in range(8)]
                ws.append(int.from_bytes(bytes(b), "little") if rng.random() < 0.7 else 0)
        segs.append(np.array(ws, dtype=np.uint64))
    return segs


def _oracle_loop(stream, limit=O.DEFAULT_TRAVERSAL_LIMIT):
    out, pos = [], 0
    while True:
        st, segs, used = O.read_message(stream[pos:], try_mode=True, limit=limit)
        if st != 0:
            return out, st
        out.append((segs, used))
        pos += used


def _check(ctx, stream, limit=O.DEFAULT_TRAVERSAL_LIMIT):
    import torch
    ref, ref_end = _oracle_loop(stream, limit)
    dev = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda() if stream else \
        torch.zeros(0, dtype=torch.uint8, device="cuda")
    got, end = ctx.read_message_stream(dev, limit=limit)
    assert end == ref_end, (end, ref_end)
    assert len(got) == len(ref), (len(got), len(ref))
    for (gsegs, gused), (rsegs, rused) in zip(got, ref):
        assert gused == rused
        assert len(gsegs) == len(rsegs)
        for a, b in zip(gsegs, rsegs):
            assert np.array_equal(a.cpu().numpy().view(np.uint64), np.asarray(b, np.uint64))


def _stream(rng, nmsg, big=False):
    out = b""
    for _ in range(nmsg):
        st, b = O.write_message(_segments(rng, big))
        assert st == 0
        out += b
    return out


def test_valid_streams(ctx):
    rng = random.Random(1)
    _check(ctx, b"")
    for nmsg in (1, 2, 5, 40, 300):
        _check(ctx, _stream(rng, nmsg))
    _check(ctx, _stream(rng, 30, big=True))


def test_truncated_and_garbage_tails(ctx):
    rng = random.Random(2)
    for trial in range(40):
        s = _stream(rng, rng.choice([1, 3, 20]))
        r = rng.random()
        if r < 0.4:
            s = s[:rng.randrange(1, len(s))]
        elif r < 0.7:
            s = s + bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
        else:
            k = rng.randrange(len(s))
            s = s[:k] + bytes([rng.choice([0, 0xFF, rng.randrange(256)])]) + s[k + 1:]
        _check(ctx, s)


def test_invalid_tables_and_limit(ctx):
    rng = random.Random(3)
    good = _stream(rng, 5)
    # segment count 0 (u32 0xFFFFFFFF + 1) and 600 segments
    bad0 = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF, 0])
    bad600 = bytes([0x03, 0x57, 0x02]) + bytes(8)
    _check(ctx, good + bad0 + good)
    _check(ctx, good + bad600)
    # a message over the traversal limit ends the loop there
    big = _stream(rng, 3, big=True)
    _check(ctx, good + big + good, limit=2000)


def test_many_tiny_messages(ctx):
    """Hundreds of 1-word (null root) and empty-segment messages: 2-4 packed
    bytes each, more than bytes // 8 + 1 of them, so discovery runs in
    several capped rounds and every message must still come back."""
    rng = random.Random(11)
    out = b""
    for k in range(700):
        segs = [np.zeros(rng.choice([0, 1]), np.uint64)]
        if k % 97 == 5:
            segs = [np.array([rng.getrandbits(64)], np.uint64)]
        st, b = O.write_message(segs)
        assert st == 0
        out += b
    assert len(out) // 8 + 1 < 700
    _check(ctx, out)
    _check(ctx, out + b"\x10\x02\x00")  # a truncated tail after them


def test_small_discovery_rounds(ctx):
    """The same loop with a cap of 3 messages per pass: ~14 passes, each
    decoding the stream again from the message after the previous pass's
    last (read_message_stream honours max_msgs)."""
    import torch
    rng = random.Random(12)
    stream = _stream(rng, 40)
    ref, ref_end = _oracle_loop(stream)
    dev = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
    got, end = ctx.read_message_stream(dev, max_msgs=3)
    assert end == ref_end and len(got) == len(ref)
    assert [u for _, u in got] == [u for _, u in ref]
    for (gs, _), (rs, _) in zip(got, ref):
        assert len(gs) == len(rs)
        for g, r in zip(gs, rs):
            assert np.array_equal(g.cpu().numpy().view(np.uint64), r)


def test_zero_heavy_stream(ctx):
    """All-zero segments expand 2 packed bytes into 256 words: the decoded
    words far exceed any fixed multiple of the packed size."""
    segs1 = [np.zeros(1 << 17, np.uint64)]                       # 1 MiB of zeros
    segs2 = [np.zeros(5000, np.uint64), np.arange(1, 9, dtype=np.uint64)]
    out = b""
    for segs in (segs1, segs2, segs1):
        st, b = O.write_message(segs)
        assert st == 0
        out += b
    assert len(out) < 10000
    _check(ctx, out)


def test_one_pass_matches_discovery(ctx):
    """decode_stream (one pass: capnp_gpu_read_message_stream) against
    find_messages + read_messages and the oracle's loop, on a stream of
    thousands of messages (hundreds of 4096-word chain ranges, messages
    longer than a range, a truncated tail): the same starts, segment tables
    and words."""
    import torch
    rng = random.Random(21)
    parts = []
    for k in range(2500):
        segs = _segments(rng, big=(k % 50 == 7))
        st, b = O.write_message(segs)
        assert st == 0
        parts.append((b, segs))
    stream = b"".join(b for b, _ in parts)
    stream_cut = stream[:-5]
    for s in (stream, stream_cut):
        dev = torch.from_numpy(np.frombuffer(s, np.uint8).copy()).cuda()
        words, mbo, bwo, segw, mso, n, clean = ctx.decode_stream(dev)
        ref, ref_end = _oracle_loop(s)
        offs, nf = ctx.find_messages(dev)
        assert clean == (ref_end == 1)
        assert n == nf and mbo.cpu().tolist() == offs.cpu().tolist()
        if s is stream:
            assert n == len(ref)
        else:
            assert n <= len(ref)
        mbo_h, bwo_h, mso_h = mbo.cpu().tolist(), bwo.cpu().tolist(), mso.cpu().tolist()
        segw_h = segw.cpu().tolist()
        w = words.cpu().numpy().view(np.uint64)
        for m in range(n):
            rsegs, rused = ref[m]
            assert mbo_h[m + 1] - mbo_h[m] == rused
            assert mso_h[m + 1] - mso_h[m] == len(rsegs)
            a = bwo_h[m]
            for j, rs in enumerate(rsegs):
                ln = segw_h[mso_h[m] + j]
                assert ln == len(rs)
                assert np.array_equal(w[a:a + ln], np.asarray(rs, np.uint64))
                a += ln


def test_truncated_inside_long_literal_run(ctx):
    """A stream cut inside a literal run that began several 512-byte blocks
    earlier: the blocks after the cut record hold no trusted chain, and the
    messages before it still come back (the complete-record prefix is found
    from the first block whose chain runs past the end)."""
    rng = random.Random(21)
    good = _stream(rng, 6)
    lit = [np.array([rng.getrandbits(64) | 0x0101010101010101 for _ in range(2000)], np.uint64)]
    st, b = O.write_message(lit)
    assert st == 0
    for cut in (40, 600, 1500, 2100, 5000, len(b) - 3):
        _check(ctx, good + b[:cut])
        _check(ctx, good + b + good[:cut % len(good)])
