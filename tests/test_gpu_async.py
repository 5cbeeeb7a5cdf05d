"""GPU parity of the streaming adaptors (capnp_packed_writer / _reader,
capnp_amd.serialize_packed_async) against the reference's async tests
(capnp-futures/src/serialize_packed.rs:560-830) and the C oracle: inputs
split at any byte, inner streams that pend and return short reads."""
import json
import os
import random

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_packing.json")))


@pytest.fixture(scope="module")
def A():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed_async as A
    return A


def check_packing_with_periods(A, rp, wp, unpacked, packed):
    # capnp-futures serialize_packed.rs:575-600
    w = A.BlockingWrite(wp)
    pw = A.PackedWrite(w)
    pw.write_all(unpacked)
    pw.flush_blocking()
    assert bytes(w.buf) == packed, (rp, wp, unpacked)
    r = A.BlockingRead(packed, rp)
    pr = A.PackedRead(r)
    assert pr.read_exact(len(unpacked)) == unpacked
    assert r.is_empty()  # nothing left to read


def test_simple_packing_blocking_periods(A):
    # simple_packing with check_packing's periods 1..9 x 1..9 (:602-671)
    for v in GOLD["packing"]:
        u, p = bytes(v["unpacked"]), bytes(v["packed"])
        for ii in range(1, 10):
            for jj in range(1, 10):
                check_packing_with_periods(A, ii, jj, u, p)


class _Plain:
    def __init__(self, data):
        self.data, self.pos = bytes(data), 0

    def read(self, n):
        b = self.data[self.pos:self.pos + n]
        self.pos += len(b)
        return b


def _read_with_size(A, n, packed, unpacked):
    # check_unpacks_with_read_size (:731-746): a plain slice reader
    pr = A.PackedRead(_Plain(packed))
    out = b""
    while len(out) < len(unpacked):
        b = pr.read(n)
        assert len(b) > 0, "premature end of stream"
        out += b
    assert out == unpacked
    assert pr.read(n) == b""


def test_unpacks_across_partial_output_buffers(A):
    _read_with_size(A, 1, bytes([0x81, 42, 99]), bytes([42, 0, 0, 0, 0, 0, 0, 99]))
    _read_with_size(A, 3, bytes([0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1]),
                    bytes([1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1]))
    # a zero run split across one-byte reads (WritingZeroes stage, :150-163)
    _read_with_size(A, 1, bytes([0, 3, 0x01, 7]), bytes(32) + bytes([7, 0, 0, 0, 0, 0, 0, 0]))


def test_eof_cases(A):
    from capnp_amd import CapnpError
    # eof_mid_tag_word (:764-777) and eof_mid_message (:805-815)
    for data in (bytes([0x81]), bytes([0xfe, 3, 3])):
        with pytest.raises(CapnpError) as e:
            A.try_read_message(_Plain(data))
        assert e.value.kind == "PrematureEndOfFile"
    # eof_mid_passthrough_run (:779-793): UnexpectedEof
    pr = A.PackedRead(_Plain(bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 2, 10, 11, 12, 13])))
    with pytest.raises(CapnpError) as e:
        pr.read_to_end()
    assert e.value.kind == "PrematureEndOfFile"
    # read_empty (:795-803)
    assert A.try_read_message(A.BlockingRead(b"", 3)) is None
    with pytest.raises(CapnpError) as e:
        A.read_message(A.BlockingRead(b"", 3))
    assert e.value.kind == "PrematureEndOfFile"


def _rand_segments(rng):
    segs = []
    for _ in range(rng.choice([1, 1, 2, 3, 5, 17])):
        n = rng.choice([0, 1, 2, 7, 40, 300])
        ws = []
        for _ in range(n):
            k = rng.random()
            if k < 0.3:
                ws.append(0)
            elif k < 0.5:
                ws.append(rng.getrandbits(64) | 0x0101010101010101)
            else:
                b = [rng.getrandbits(8) if rng.random() < 0.6 else 0 for _ in range(8)]
                ws.append(int.from_bytes(bytes(b), "little"))
        segs.append(np.array(ws, dtype=np.uint64))
    return segs


def test_round_trip_async_periods(A):
    # round_trip / check_packed_round_trip_async (:673-729): write_message
    # through a blocking writer, try_read_message through a blocking reader;
    # the bytes equal the sync writer's (overflow_test.rs:65-79)
    rng = random.Random(5)
    cases = [[np.array([int.from_bytes(bytes([8, 14, 90, 7, 21, 13, 59, 17]), "little"),
                        int.from_bytes(bytes([0, 31, 21, 73, 0, 54, 61, 12]), "little")],
                       dtype=np.uint64)]]  # check_packed_round_trip_async_bug
    cases += [_rand_segments(rng) for _ in range(40)]
    for i, segs in enumerate(cases):
        rp, wp = rng.randrange(1, 12), rng.randrange(1, 12)
        w = A.BlockingWrite(wp)
        A.write_message(w, segs)
        st, ref = O.write_message(segs)
        assert st == 0 and bytes(w.buf) == ref, i
        r = A.BlockingRead(bytes(w.buf), rp)
        got = A.try_read_message(r)
        assert len(got) == len(segs)
        for a, b in zip(got.segments(), segs):
            assert np.array_equal(np.asarray(a).view(np.uint64), b)
        assert r.is_empty()


def _split_points(rng, n):
    pts, k = [], 0
    while k < n:
        k = min(n, k + rng.choice([1, 2, 3, 5, 7, 8, 9, 15, 16, 17, 64, 1000]))
        pts.append(k)
    return pts


def _async_write_model(data, pts):
    """The async writer's chunks for write calls ending at `pts`: a word
    completed from carried bytes plus this call's whole words, packed as one
    write_all (serialize_packed.rs:370-452 of capnp-futures)."""
    out, carry, a = b"", b"", 0
    for b in pts:
        buf = carry + data[a:b]
        m = len(buf) // 8
        if m:
            st, p = O.pack(buf[:8 * m])
            assert st == 0
            out += p
        carry = buf[8 * m:]
        a = b
    return out, carry


def test_writes_split_at_any_byte(A):
    rng = random.Random(11)
    for trial in range(60):
        segs = _rand_segments(rng)
        data = b"".join(s.tobytes() for s in segs)
        if not data:
            continue
        pts = _split_points(rng, len(data))
        w = A.BlockingWrite(rng.randrange(1, 9))
        pw = A.PackedWrite(w)
        a = 0
        for b in pts:
            pw.write(data[a:b])
            a = b
        pw.flush_blocking()
        ref, carry = _async_write_model(data, pts)
        assert bytes(w.buf) == ref, trial
        assert pw.carried == len(carry) == 0
        # reads of any size give the bytes back
        pr = A.PackedRead(A.BlockingRead(ref, rng.randrange(1, 9)))
        out = b""
        while True:
            try:
                b = pr.read(rng.choice([1, 3, 8, 13, 64, 4096]))
            except Exception as e:
                if getattr(e, "status", None) == 15:
                    continue
                raise
            if not b:
                break
            out += b
        assert out == data, trial


def test_partial_word_carried(A):
    w = A.BlockingWrite(1 << 30)
    pw = A.PackedWrite(w)
    pw.write(bytes([1, 2, 3]))
    assert pw.carried == 3
    pw.flush_blocking()
    assert bytes(w.buf) == b""  # an incomplete word is not emitted
    pw.write(bytes([4, 5, 6, 7, 8]) + bytes(16))
    pw.flush_blocking()
    st, ref = O.pack(bytes([1, 2, 3, 4, 5, 6, 7, 8]) + bytes(16))
    assert bytes(w.buf) == ref and pw.carried == 0


def test_message_stream_try_read_loop(A):
    # a concatenated stream read message by message until try_read_message
    # returns None (serialize.rs:310-325 via the async twin)
    rng = random.Random(3)
    msgs = [_rand_segments(rng) for _ in range(25)]
    stream = b""
    for segs in msgs:
        st, b = O.write_message(segs)
        stream += b
    r = A.BlockingRead(stream, 97)
    pr = A.PackedRead(r)
    got = []
    while True:
        m = A.try_read_message(pr)
        if m is None:
            break
        got.append(m)
    assert len(got) == len(msgs)
    for m, segs in zip(got, msgs):
        for a, b in zip(m.segments(), segs):
            assert np.array_equal(np.asarray(a).view(np.uint64), b)


# ---- sync PackedRead over a BufRead that refills (io.rs:35-38,
# refresh_buffer! serialize_packed.rs:59-74)

class _Raw:
    def __init__(self, data):
        self.data, self.pos = bytes(data), 0

    def read(self, n):
        b = self.data[self.pos:self.pos + n]
        self.pos += len(b)
        return b


def test_bufread_refill_messages():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed as S
    rng = random.Random(21)
    msgs = [_rand_segments(rng) for _ in range(20)]
    stream = b""
    for segs in msgs:
        st, b = O.write_message(segs)
        stream += b
    for cap in (7, 64, 1000, 1 << 16):
        r = S.BufReader(_Raw(stream), capacity=cap)
        for segs in msgs:
            m = S.try_read_message(r)
            assert m is not None and len(m) == len(segs), cap
            for a, b in zip(m.segments(), segs):
                assert np.array_equal(np.asarray(a).view(np.uint64), b), cap
        assert S.try_read_message(r) is None, cap
    # a message cut short: the error is the one the whole input gives
    cut = stream[:len(stream) // 3]
    ref_st = None
    pos = 0
    while True:
        st, segs_, used = O.read_message(cut[pos:], try_mode=True)
        if st != 0:
            ref_st = st
            break
        pos += used
    from capnp_amd import CapnpError
    r = S.BufReader(_Raw(cut), capacity=50)
    with pytest.raises(CapnpError) as e:
        while S.try_read_message(r) is not None:
            pass
    assert e.value.status == ref_st


def test_bufread_refill_read_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed as S
    for v in GOLD["packing"]:
        u, p = bytes(v["unpacked"]), bytes(v["packed"])
        if not u:
            continue
        for cap in (1, 2, 3, 9, 100):
            r = S.BufReader(_Raw(p + b"\x07\x07"), capacity=cap)
            assert S.PackedRead(r).read_exact(len(u)) == u
            # the bytes after the unit stay unread
            rest = b""
            while True:
                b = bytes(r.fill_buf())
                if not b:
                    break
                rest += b
                r.consume(len(b))
            assert rest == b"\x07\x07", (cap, v)


class _PlainBufRead:
    """A minimal BufRead (fill_buf / consume only), as a Rust caller's
    reader: the streamed read units (serialize_packed._read_unit) need
    nothing more."""

    def __init__(self, raw, capacity):
        self.raw, self.capacity, self.buf, self.pos = raw, capacity, b"", 0

    def fill_buf(self):
        if self.pos >= len(self.buf):
            self.buf, self.pos = bytes(self.raw.read(self.capacity)), 0
        return memoryview(self.buf)[self.pos:]

    def consume(self, n):
        self.pos = min(self.pos + n, len(self.buf))


def _drain(r):
    rest = b""
    while True:
        b = bytes(r.fill_buf())
        if not b:
            return rest
        rest += b
        r.consume(len(b))


def test_bufread_lookahead_stops_where_reference_does():
    """Over BufReader and a minimal BufRead alike, at buffer sizes from 5
    bytes to 4 KiB, the reader returns the same messages and error and
    leaves the same bytes; after each message exactly the bytes the oracle's
    read_message used are gone."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed as S
    from capnp_amd import CapnpError
    rng = random.Random(23)
    stream = b""
    for _ in range(12):
        st, b = O.write_message(_rand_segments(rng))
        stream += b
    cases = [stream, stream[:len(stream) * 2 // 3], stream + b"\x00\x05",
             stream[:200] + b"\xff\x01\x02", stream + bytes([0xff] + [7] * 8 + [3])]
    for data in cases:
        for cap in (5, 33, 256, 4096):
            res = []
            for mk in (lambda: S.BufReader(_Raw(data), capacity=cap),
                       lambda: _PlainBufRead(_Raw(data), cap)):
                r = mk()
                got, err = [], None
                try:
                    while True:
                        m = S.try_read_message(r)
                        if m is None:
                            break
                        got.append([np.asarray(s).view(np.uint64).tobytes()
                                    for s in m.segments()])
                except CapnpError as e:
                    err = e.status
                res.append((got, err, _drain(r)))
            assert res[0] == res[1], (cap, len(data))
            # the messages and where the reader stands after them, against
            # the oracle's read_message loop
            pos, ref = 0, []
            while True:
                st_, segs_, used_ = O.read_message(data[pos:], try_mode=True)
                if st_ != 0:
                    break
                ref.append([np.asarray(x, np.uint64).tobytes() for x in segs_])
                pos += used_
            assert res[0][0] == ref, cap
            if res[0][1] is None:
                assert res[0][2] == b"" and pos == len(data), cap


def test_bufread_large_message_small_buffer():
    """An 8 MiB message through 8 KiB buffers (1024 refills): each buffer
    is decoded once (the streamed units carry only an incomplete record)."""
    import time
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed as S
    words = O.gen_fill(np.array([0, 1 << 20], np.uint64))
    st, b = O.write_message([words])
    assert st == 0
    r = S.BufReader(_Raw(b + b"\x01\x02\x03"), capacity=8192)
    t0 = time.perf_counter()
    m = S.read_message(r, S.ReaderOptions(traversal_limit_in_words=None))
    dt = time.perf_counter() - t0
    assert np.array_equal(np.asarray(m.get_segment(0)).view(np.uint64), words)
    assert _drain(r) == b"\x01\x02\x03"
    assert dt < 30, dt


def test_async_reader_inner_overread():
    """An inner reader that returns more bytes than asked: the adaptor takes
    only what fits and keeps the rest for the next pull."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import serialize_packed_async as A
    u = bytes(range(1, 65)) * 64
    st, p = O.pack(u)
    assert st == 0

    class Greedy:
        def __init__(self, data):
            self.data, self.pos = data, 0

        def read(self, n):
            b = self.data[self.pos:self.pos + 2 * n + 7]  # more than asked
            self.pos += len(b)
            return b

    r = A.PackedRead(Greedy(p))
    got = b""
    while len(got) < len(u):
        b = r.read(len(u) - len(got))
        assert b
        got += b
    assert got == u


def _ref_poll_reads(packed, size, inner_max=1 << 30):
    """The oracle's restatement of capnp-futures PackedRead::poll_read
    (oracle/packed_ref.py async_poll_reads, pinned by the reference's async
    test vectors in tests/test_oracle.py)."""
    import packed_ref
    return packed_ref.async_poll_reads(packed, size, inner_max)


def test_partial_delivery_before_eof(A):
    """Truncated streams read in 1-, 3- and 8-byte reads: the bytes handed
    out before the error (or the clean end) are those of the reference's
    stage machine: a literal run's head word and whatever raw bytes arrived
    come out before UnexpectedEof (eof_mid_passthrough_run, :779-793)."""
    from capnp_amd import CapnpError
    lit = bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 2, 10, 11, 12, 13])
    st_, full = O.pack(bytes([9, 0, 3, 0, 0, 0, 0, 1]) + bytes(range(1, 33)) * 4 + bytes(24)
                       + bytes(range(2, 26)))
    cases = [lit, lit[:9], lit[:10], lit[:11], bytes([0x81]), bytes([0xfe, 3, 3]), bytes([0]),
             bytes([0, 3]), bytes([0x81, 42, 99]), lit + bytes(12)]
    cases += [full[:k] for k in range(len(full) + 1)]
    for data in cases:
        for size in (1, 3, 8):
            ref, end = _ref_poll_reads(data, size)
            pr = A.PackedRead(_Plain(data))
            got, err = b"", None
            while True:
                try:
                    b = pr.read(size)
                except CapnpError as e:
                    err = e.kind
                    break
                if not b:
                    break
                assert len(b) <= size
                got += b
            assert got == ref, (data, size, got, ref)
            assert (err == "PrematureEndOfFile") == (end == "EOF"), (data, size, err, end)


def test_literal_head_while_pending(A):
    """An inner reader that pends inside a literal run's raw words: the head
    word is handed out at once (the reference's DrainingBuffer stage), the
    raw bytes pass through as they arrive."""
    from capnp_amd import CapnpError
    lit = bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 2]) + bytes(range(10, 26))

    class Trickle:
        """The first 12 bytes, then pending once, then the rest."""
        def __init__(self, data):
            self.data, self.pos, self.pended = data, 0, False

        def read(self, n):
            if self.pos == 12 and not self.pended:
                self.pended = True
                return None
            end = 12 if self.pos < 12 else len(self.data)
            b = self.data[self.pos:min(end, self.pos + n)]
            self.pos += len(b)
            return b

    pr = A.PackedRead(Trickle(lit))
    got = b""
    pends = 0
    while len(got) < 24:
        try:
            b = pr.read(24 - len(got))
        except CapnpError as e:
            assert e.status == 15  # pending
            pends += 1
            continue
        assert b
        got += b
        if len(got) == 10:
            assert pends == 0  # head word + 2 raw bytes before the inner reader pended
    assert got == bytes(range(1, 9)) + bytes(range(10, 26))
    assert pends <= 1  # (the pend may be absorbed while the head word is decoded)
    assert pr.read(8) == b""


def _mixed_words(seed, n):
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    w[rng.random(n) < 0.3] = 0
    w[n // 7:n // 7 + 3000] = 0  # long zero runs
    w[n // 3:n // 3 + 4000] |= np.uint64(0x0101010101010101)  # long literal runs
    sparse = rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(8 * 3)
    w[n // 2:n // 2 + 5000] = sparse[:5000]
    return w


def test_large_reads_whole_records(A):
    """Reads of 64 KiB and more take whole-record units resolved on the
    device (stream_io.hip reader_fill_whole): every read returns 1..n bytes,
    the bytes are the stream's, a plain and a pending inner reader alike."""
    from capnp_amd import CapnpError
    w = _mixed_words(7, 300_000)
    u = w.tobytes()
    st, p = O.pack(u)
    assert st == 0
    for size in (1 << 20, (1 << 16) + 8, 200_008):
        for inner in (_Plain(p), A.BlockingRead(p, 70_001)):
            pr = A.PackedRead(inner)
            got = bytearray()
            while True:
                try:
                    b = pr.read(size)
                except CapnpError as e:
                    assert e.status == 15  # pending
                    continue
                if not b:
                    break
                assert 0 < len(b) <= size
                got += b
            assert bytes(got) == u, size


def test_large_reads_truncated_stream(A):
    """A truncated stream read in 1 MiB reads hands out what the reference's
    stage machine does before UnexpectedEof (whole records, then a literal
    run's head word and raw bytes)."""
    from capnp_amd import CapnpError
    w = _mixed_words(8, 40_000)
    st, p = O.pack(w.tobytes())
    assert st == 0
    for cut in (len(p) - 1, len(p) - 5, len(p) // 3 + 17, len(p) // 3 + 1000, len(p) // 2 + 1,
                len(p) // 7 + 3):
        data = p[:cut]
        ref, end = _ref_poll_reads(data, 1 << 20)
        pr = A.PackedRead(_Plain(data))
        got, err = b"", None
        while True:
            try:
                b = pr.read(1 << 20)
            except CapnpError as e:
                err = e.kind
                break
            if not b:
                break
            got += b
        assert got == ref, (cut, len(got), len(ref))
        assert (err == "PrematureEndOfFile") == (end == "EOF"), (cut, err, end)


class _Pipe:
    """A blocking pipe after the peer wrote `data` and waits for an answer:
    a read returns what is buffered (short reads, POSIX read(2)), and a read
    with nothing buffered would block forever -- here it fails the test."""

    def __init__(self, data, piece=None):
        self.data, self.pos, self.piece = bytes(data), 0, piece
        self.reads = 0

    def read(self, n):
        if self.pos == len(self.data):
            raise AssertionError("read() on an empty blocking pipe: would hang")
        k = min(n, len(self.data) - self.pos, self.piece or n)
        self.reads += 1
        b = self.data[self.pos:self.pos + k]
        self.pos += k
        return b


@pytest.mark.parametrize("body_words,piece", [(200, None), (20_000, None), (300_000, None),
                                              (300_000, 65_536 + 24)])
def test_reader_stops_at_request_over_blocking_pipe(A, body_words, piece):
    """read_message over a blocking inner reader that has exactly one message
    buffered returns that message without another read (the reference's
    PackedRead pulls only what the caller's words need): no read-ahead of MiBs
    on the caller's thread (stream_io.hip reader_ahead)."""
    rng = np.random.default_rng(body_words)
    seg = rng.integers(0, 1 << 63, body_words, dtype=np.uint64)
    seg[rng.random(body_words) < 0.3] = 0
    st, msg = O.write_message([seg])
    assert st == 0
    pipe = _Pipe(msg, piece)
    pr = A.PackedRead(pipe)
    m = A.read_message(pr)
    assert np.array_equal(np.asarray(m.segments()[0]).view(np.uint64), seg)
    assert pipe.pos == len(msg)


@pytest.mark.parametrize("total", [1 << 16, 1 << 17, 3 << 16])
def test_reader_no_pull_past_full_request(A, total):
    """A blocking peer that sent exactly a multiple of the adaptor's pull size
    (64 KiB) and now awaits a reply: the reads that the staged bytes can
    serve are served without another pull (stream_io.hip: a pull
    that came back full no longer licenses a pull past the request)."""
    # one message of 1-byte words (2 packed bytes each) padded to `total`
    n = (total - 16) // 2
    for k in range(n, n - 64, -1):
        seg = np.ones(k, np.uint64)
        st, msg = O.write_message([seg])
        assert st == 0
        if len(msg) <= total and (total - len(msg)) % 3 == 0:
            break
    extra = (total - len(msg)) // 3  # words of 2 nonzero bytes: 3 packed bytes each
    seg = np.ones(k + extra, np.uint64)
    seg[:extra] = 0x0101
    st, msg = O.write_message([seg])
    assert st == 0 and len(msg) == total, (len(msg), total)
    pipe = _Pipe(msg, None)
    pr = A.PackedRead(pipe)
    m = A.read_message(pr)
    assert np.array_equal(np.asarray(m.segments()[0]).view(np.uint64), seg)
    assert pipe.pos == len(msg)


def test_writer_list_sink_keeps_its_bytes(A):
    """An inner writer that keeps what it is given (no copy) sees bytes that
    stay valid after the adaptor reuses its queue."""
    class Keep:
        def __init__(self):
            self.parts = []

        def write(self, b):
            self.parts.append(b)  # (keeps the object itself)
            return len(b)

    w = _mixed_words(11, 150_000)
    u = w.tobytes()
    sink = Keep()
    pw = A.PackedWrite(sink)
    for i in range(0, len(u), 1 << 18):
        pw.write_all(u[i:i + (1 << 18)])
        pw.flush_blocking()
    ref = b""
    for i in range(0, len(u), 1 << 18):
        ref += O.pack(u[i:i + (1 << 18)])[1]
    assert b"".join(bytes(x) for x in sink.parts) == ref


def test_reader_reused_bytearray(A):
    """An inner reader that returns its own reused bytearray: the bytes the
    adaptor carries past one call are its own copy."""
    w = _mixed_words(12, 60_000)
    u = w.tobytes()
    st, p = O.pack(u)

    class Reuse:
        def __init__(self, data):
            self.data, self.pos, self.buf = data, 0, bytearray(100_003)

        def read(self, n):
            k = min(len(self.buf), len(self.data) - self.pos)
            self.buf[:k] = self.data[self.pos:self.pos + k]
            self.pos += k
            return memoryview(self.buf)[:k]

    pr = A.PackedRead(Reuse(p))
    got = bytearray()
    while True:
        b = pr.read(4096)
        if not b:
            break
        got += b
    assert bytes(got) == u
