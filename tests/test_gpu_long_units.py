"""GPU parity of the long-unit decode (csrc/unpack.hip unpack_long: a chunk
too large for the tile tables, decoded by the whole workgroup in 16 KiB
windows; msg_read_kernel decodes read_message bodies with it) against the
oracle's read_exact (serialize_packed.rs:80-228, io.rs:16-31).

Pins the round-4 r04g2 failure's boundary: a read_message body on the global
path came back all zero (tests/test_gpu_async.py::test_bufread_refill_messages
at a 64 KiB BufReader), in a build whose window refill of the serial walk
(unpack_global1) bounded its 16-byte vector loads by the chunk end without
the start's misalignment -- so with a body starting mis bytes past a 16-byte
boundary, the vectors holding its last mis bytes were zero-filled and read as
zero-run records.  Here: long units starting at every misalignment 0..15,
ending at every offset of a vector, with spare bytes after (a stream's next
message), through the batch path and through read_message; malformed units
at the same starts take the exact serial walk (the fallback) and must give
the oracle's status and consumed count."""
import ctypes as C

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


def _unit(words, kind, seed):
    offs = np.array([0, words], np.uint64)
    w = O.gen_fill(offs, kinds=np.array([kind], np.uint8), pz=O.PZ30, id0=seed)
    st, p = O.pack(w.tobytes())
    assert st == 0
    return w, np.frombuffer(p, np.uint8)


def _decode(ctx, buf, a, b, n):
    """One chunk [a, b) of buf, n words, chunks_per_tile=1 (the overflow path)."""
    dev = torch.device("cuda", 0)
    packed = torch.from_numpy(buf.copy()).to(dev)
    inoff = torch.tensor([a, b], dtype=torch.int64, device=dev)
    outoff = torch.tensor([0, n], dtype=torch.int64, device=dev)
    words = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)
    st = torch.full((1,), -1, dtype=torch.int32, device=dev)
    used = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.unpack_batch_into(packed, inoff, outoff, words, st, used, chunks_per_tile=1)
    torch.cuda.synchronize()
    return (words.cpu().numpy().view(np.uint64)[:n], int(st.cpu()[0]), int(used.cpu()[0]))


@pytest.mark.parametrize("kind", [0, 2])
def test_long_unit_every_misalignment(ctx, kind):
    w, p = _unit(3000 if kind == 0 else 2600, kind, 40 + kind)
    n = len(w)
    spare = _unit(64, 0, 99)[1]
    for mis in range(16):
        buf = np.concatenate([np.full(mis, 0xA5, np.uint8), p, spare, np.zeros(32, np.uint8)])
        a, b = mis, mis + len(p) + len(spare)  # (spare bytes: the decode stops after n words)
        got, st, used = _decode(ctx, buf, a, b, n)
        rst, rb, rused = O.read_exact(bytes(buf[a:b]), n * 8)
        assert st == rst == 0 and used == rused == len(p), mis
        assert np.array_equal(got, w), mis


def test_long_unit_every_end_offset(ctx):
    # units whose packed end falls on each offset of a 16-byte vector, no spare
    for k in range(16):
        w, p = _unit(2100 + 7 * k, 0, 60 + k)
        for mis in (0, 5, 15):
            buf = np.concatenate([np.zeros(mis, np.uint8), p, np.zeros(32, np.uint8)])
            got, st, used = _decode(ctx, buf, mis, mis + len(p), len(w))
            assert st == 0 and used == len(p), (k, mis)
            assert np.array_equal(got, w), (k, mis)


def test_long_unit_malformed_serial_fallback(ctx):
    # truncated (PrematureEnd / FailedToFill), a run past the words
    # (DidNotEndCleanly) and too few bytes: the exact serial walk's statuses
    w, p = _unit(3000, 0, 77)
    wl, pl = _unit(2600, 2, 78)
    cases = [(p[:len(p) - 1], len(w)), (p[:len(p) // 2], len(w)), (p, len(w) - 1),
             (pl[:len(pl) - 100], len(wl)), (pl, len(wl) - 3), (p, len(w) + 5)]
    for mis in (0, 3, 11):
        for data, n in cases:
            buf = np.concatenate([np.zeros(mis, np.uint8), data, np.zeros(32, np.uint8)])
            got, st, used = _decode(ctx, buf, mis, mis + len(data), n)
            rst, rb, rused = O.read_exact(bytes(data), n * 8)
            assert (st, used) == (rst, rused), (mis, len(data), n)


def test_read_message_long_bodies_misaligned(ctx):
    """read_message (one launch: msg_read_kernel) of messages whose body is
    on the long-unit path, tables of 1..6 segments (so the body starts at
    several misalignments), the next message's bytes after it."""
    from capnp_amd import _lib
    L = _lib.lib()
    opts = _lib.ReaderOptionsC(0, 0, 64)
    rng = np.random.default_rng(5)
    for nseg in range(1, 7):
        segs = []
        for i in range(nseg):
            k = int(rng.integers(1, 2600))
            offs = np.array([0, k], np.uint64)
            segs.append(O.gen_fill(offs, kinds=np.array([i % 3], np.uint8), pz=O.PZ30,
                                   id0=300 + 10 * nseg + i))
        st, msg = O.write_message(segs)
        st2, nxt = O.write_message([segs[0][:5]])
        data = np.frombuffer(msg + nxt, np.uint8).copy()
        total = sum(len(s) for s in segs)
        body = np.zeros(total + 1, np.uint64)
        sw = np.zeros(512, np.uint32)
        ns, used = C.c_uint32(0), C.c_size_t(0)
        r = L.capnp_packed_read_message(ctx.handle, data.ctypes.data, len(data), C.byref(opts),
                                        0, body.ctypes.data, total + 1, sw.ctypes.data,
                                        C.byref(ns), C.byref(used))
        rst, rsegs, rused = O.read_message(bytes(data))
        assert r == rst == 0 and used.value == rused == len(msg), nseg
        assert ns.value == nseg
        o = 0
        for s in segs:
            assert np.array_equal(body[o:o + len(s)], s), nseg
            o += len(s)


def _batch(ctx, units, mis=0, resync=False, cpt=0):
    """Chunks back to back (mis junk bytes first); returns per-chunk words,
    statuses and consumed counts from the batch (or index-free) decode."""
    dev = torch.device("cuda", 0)
    parts = [np.full(mis, 0x5A, np.uint8)] + [p for _, p, _ in units] + [np.zeros(32, np.uint8)]
    buf = np.concatenate(parts)
    inoff = np.cumsum([mis] + [len(p) for _, p, _ in units]).astype(np.int64)
    outoff = np.cumsum([0] + [n for _, _, n in units]).astype(np.int64)
    packed = torch.from_numpy(buf).to(dev)
    ti = torch.from_numpy(inoff).to(dev)
    to = torch.from_numpy(outoff).to(dev)
    words = torch.zeros(max(int(outoff[-1]), 1), dtype=torch.int64, device=dev)
    st = torch.full((len(units),), -1, dtype=torch.int32, device=dev)
    used = torch.zeros(len(units), dtype=torch.int64, device=dev)
    if resync:
        ctx.unpack_batch_resync_into(packed, ti, to, words, st, used)
    else:
        ctx.unpack_batch_into(packed, ti, to, words, st, used, chunks_per_tile=cpt)
    torch.cuda.synchronize()
    return words.cpu().numpy().view(np.uint64), st.cpu().numpy(), used.cpu().numpy(), outoff


@pytest.mark.parametrize("resync", [False, True])
def test_big_staged_units_batch(ctx, resync):
    """Overflow chunks of 2049..8192 words and <= 16 KiB packed take the
    staged decode with the 8192-word / 16 KiB tables inside the long-unit LDS
    (unpack.hip BigStageSmem); past either limit they take unpack_long.  Units
    on both sides of both limits, zero-heavy (kind 1: 8192 and 8193 words,
    a few hundred packed bytes) and literal-heavy ones, interleaved with short
    chunks, plus malformed ones, against read_exact per chunk."""
    rng = np.random.default_rng(11)
    spec = [(2049, 0), (3800, 0), (3900, 0), (8192, 1), (8193, 1), (12000, 1),
            (2040, 2), (2060, 2), (5000, 1), (64, 0), (7, 2), (8191, 1), (3000, 0)]
    units = []
    for i, (n, kind) in enumerate(spec):
        w, p = _unit(n, kind, 500 + i)
        units.append((w, p, n))
    # malformed: a truncated big-path unit, a zero-heavy unit one word short
    # (its last zero run overruns: DidNotEndCleanly), a literal-heavy cut
    wb, pb = _unit(3000, 0, 601)
    wz, pz = _unit(6000, 1, 602)
    wl, pl = _unit(2030, 2, 603)
    bad = [(wb, pb[:len(pb) - 37], 3000), (wz, pz, 5999), (wl, pl[:len(pl) // 2], 2030)]
    for order in (units, units + bad, bad[:1] + units[::-1]):
        for mis in (0, 9):
            got, st, used, outoff = _batch(ctx, order, mis, resync)
            for k, (w, p, n) in enumerate(order):
                rst, rb, rused = O.read_exact(bytes(p), n * 8)
                assert (int(st[k]), int(used[k])) == (rst, rused), (k, n, mis)
                if rst == 0:
                    assert np.array_equal(got[outoff[k]:outoff[k + 1]], w), (k, n, mis)


@pytest.mark.parametrize("n,kind", [(8192, 1), (8193, 1), (3800, 0), (4000, 0), (10000, 0)])
def test_big_and_long_unit_misaligned(ctx, n, kind):
    """One chunk at each start misalignment 0..15 on both sides of the
    staged-path limits (8192 words; 16 KiB packed: kind 0 crosses it between
    3800 and 4000 words) with the next chunk's bytes after it."""
    w, p = _unit(n, kind, 700 + n)
    spare = _unit(64, 2, 98)[1]
    for mis in range(16):
        buf = np.concatenate([np.full(mis, 0xC3, np.uint8), p, spare, np.zeros(32, np.uint8)])
        got, st, used = _decode(ctx, buf, mis, mis + len(p) + len(spare), n)
        rst, rb, rused = O.read_exact(bytes(buf[mis:mis + len(p) + len(spare)]), n * 8)
        assert st == rst == 0 and used == rused == len(p), mis
        assert np.array_equal(got, w), mis



def _read_message_call(handle, data):
    from capnp_amd import _lib
    L = _lib.lib()
    opts = _lib.ReaderOptionsC(0, 0, 64)
    data = np.frombuffer(bytes(data), np.uint8).copy()
    cap = len(data) * 128 + 64
    body = np.zeros(cap + 1, np.uint64)
    sw = np.zeros(512, np.uint32)
    ns, used = C.c_uint32(0), C.c_size_t(0)
    r = L.capnp_packed_read_message(handle, data.ctypes.data, len(data), C.byref(opts), 0,
                                    body.ctypes.data, cap + 1, sw.ctypes.data, C.byref(ns),
                                    C.byref(used))
    return r, body, used.value


def _packed(words):
    st, b = O.pack(np.asarray(words, np.uint64).tobytes())
    assert st == 0
    return b


def test_read_message_small_bodies_vs_oracle(ctx):
    """read_message's short bodies (csrc/unpack.hip unpack_small: wave 0
    alone, 64 segments, inside the staged prefix) against the oracle's
    read_message: valid bodies of 1..1600 words of every fill kind, alone
    and with the next message's bytes after them; truncated inputs; tables
    claiming fewer words than the body's records cover (the last run
    overruns); random bytes after a valid table -- status, consumed bytes
    and the segment words."""
    rng = np.random.default_rng(21)
    cases = []
    for k in (1, 2, 7, 64, 65, 128, 300, 777, 1500, 1600):
        for kind in (0, 1, 2):
            w = O.gen_fill(np.array([0, k], np.uint64), kinds=np.array([kind], np.uint8),
                           pz=O.PZ30, id0=900 + k + kind)
            st, msg = O.write_message([w])
            assert st == 0 and msg == _packed([k << 32]) + _packed(w)
            cases.append(msg)
            cases.append(msg + O.write_message([w[:3]])[1])  # the next message follows
            cases.append(msg[:len(msg) - 1])                  # truncated by a byte
            cases.append(msg[:max(9, len(msg) // 2)])         # truncated in the body
            if k > 1:  # the table claims one word fewer than the records cover
                cases.append(_packed([(k - 1) << 32]) + _packed(w))
    for i in range(40):  # a valid one-segment table, then random body bytes
        k = int(rng.integers(1, 400))
        body = rng.integers(0, 256, int(rng.integers(1, 12 * k))).astype(np.uint8).tobytes()
        cases.append(_packed([k << 32]) + body)
    for data in cases:
        rst, rsegs, rused = O.read_message(bytes(data))
        r, body, used = _read_message_call(ctx.handle, data)
        assert r == rst, (len(data), r, rst)
        if rst == 0:
            assert used == rused, (len(data), used, rused)
            o = 0
            for sgm in rsegs:
                assert np.array_equal(body[o:o + len(sgm)], sgm)
                o += len(sgm)


def test_read_message_mid_bodies_vs_oracle(ctx):
    """read_message's mid-size bodies (csrc/unpack.hip unpack_mid: bodies of
    5-18 KB packed inside the staged prefix, four waves of 64 segments that
    settle by themselves and meet through LDS) against the oracle's
    read_message: every fill kind at sizes around both edges (the short-body
    path below 5 KB, the long-unit decode above 18 KB), with the next
    message after them, truncated by a byte and inside the body, tables
    claiming fewer words than the records cover, literal runs and zero runs
    across the waves' quarters, a flipped byte, and random bytes after a
    valid table -- status, consumed bytes and the segment words."""
    rng = np.random.default_rng(33)
    cases = []
    for k in (560, 600, 700, 900, 1024, 1500, 1800, 2000, 2200, 2400, 3600, 4096, 4300, 8192):
        for kind in (0, 1, 2):
            w = O.gen_fill(np.array([0, k], np.uint64), kinds=np.array([kind], np.uint8),
                           pz=O.PZ30, id0=1900 + k + kind)
            st, msg = O.write_message([w])
            assert st == 0
            cases.append(msg)
            cases.append(msg + O.write_message([w[:3]])[1])
            cases.append(msg[:len(msg) - 1])
            cases.append(msg[:max(9, len(msg) // 2)])
            cases.append(_packed([(k - 1) << 32]) + _packed(w))
            bad = bytearray(msg)
            bad[8 + int(rng.integers(0, len(msg) - 8))] ^= 0x5A
            cases.append(bytes(bad))
    # runs crossing the quarter cuts: literal words then zeros then literal
    for k in (800, 1500, 2000):
        w = np.zeros(k, np.uint64)
        a, b = k // 4 - 7, k // 2 + 5
        w[:a] = 0x0102030405060708
        w[b:] = 0x1112131415161718
        w[rng.integers(0, k, 5)] = 0x0000000400000001
        cases.append(O.write_message([w])[1])
    for i in range(30):  # a valid one-segment table, then random body bytes
        k = int(rng.integers(500, 2000))
        body = rng.integers(0, 256, int(rng.integers(5200, 16000))).astype(np.uint8).tobytes()
        cases.append(_packed([k << 32]) + body)
    for data in cases:
        rst, rsegs, rused = O.read_message(bytes(data))
        r, body, used = _read_message_call(ctx.handle, data)
        assert r == rst, (len(data), r, rst)
        if rst == 0:
            assert used == rused, (len(data), used, rused)
            o = 0
            for sgm in rsegs:
                assert np.array_equal(body[o:o + len(sgm)], sgm)
                o += len(sgm)
