"""GPU parity at the size thresholds that pick a code path (VERDICT r05,
weak #1): each side of every edge against the oracle.

* write_message (capnp_packed_write_message, csrc/capi.hip): the one-launch
  kernel (msg_pack_kernel) takes messages of <= capnp_msg_pack_words()
  (8448) words and <= 515 chunks; past that the pinned mid-size path, and
  past kWritePinMax (4 MiB staged) the pageable path.
  Reference: serialize.rs:574-679, serialize_packed.rs:446-453.
* read_message (capnp_packed_read_message): bodies under
  PARALLEL_BODY_WORDS (65536) decode in one launch (msg_read_kernel), longer
  ones through the index-free block decode; each size also truncated by one
  byte.  Reference: serialize.rs:448-524, serialize_packed.rs:233-255.
"""
import random

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_long_units import _read_message_call
from test_gpu_parity import _rand_segment, _runs_segment

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MSG_WORDS = 8448          # capnp_msg_pack_words() (pack.hip kMsgWords)
MSG_CHUNKS = 515          # the one-launch chunk limit (capi.hip)
PIN_MAX = 4 << 20         # kWritePinMax (capi.hip)
BODY_WORDS = 65536        # PARALLEL_BODY_WORDS (capi.hip)


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


def _table_words(nseg):
    rest = 0 if nseg == 1 else (8 if nseg < 4 else (nseg & ~1) * 4)
    return 1 + rest // 8


def _write_check(ctx, segs, what):
    from capnp_amd import serialize_packed as sp
    out = bytearray()
    sp.write_message(out, segs, ctx=ctx)
    st, ref = O.write_message(segs)
    assert st == 0 and bytes(out) == ref, what
    return ref


def test_msg_pack_kernel_word_edge(ctx):
    """One segment (1 table word) and two segments (2 table words) whose
    message is 8447, 8448 (the last one-launch size) and 8449 words; the long
    segment built from runs across the kernel's 64-word wave ranges, and plain
    mixed data."""
    from capnp_amd import _lib
    assert _lib.lib().capnp_msg_pack_words() == MSG_WORDS
    rng = random.Random(606)
    for nw in (MSG_WORDS - 1, MSG_WORDS, MSG_WORDS + 1):
        for gen in (_runs_segment, _rand_segment):
            _write_check(ctx, [gen(rng, nw - 1)], ("1 seg", nw, gen.__name__))
            a = rng.choice([1, 63, 64, 65, 500])
            _write_check(ctx, [gen(rng, a), gen(rng, nw - 2 - a)], ("2 segs", nw, a))
    # the last segment ending exactly on a 64-word wave split, and one word short
    for tail in (0, 1, 63):
        n = (MSG_WORDS - 1) // 64 * 64 - tail
        _write_check(ctx, [_runs_segment(rng, n)], ("split end", n))


def test_msg_pack_kernel_chunk_edge(ctx):
    """513 segments (515 chunks: word 0, table rest, segments; the last
    one-launch count) and 514 (516), with the message words well inside the
    word limit; also 511 (the most a reader accepts, serialize.rs:467-473)
    for the round trip."""
    from capnp_amd import serialize_packed as sp
    rng = random.Random(515)
    for nseg in (511, 512, 513, 514):
        nch = 2 + nseg
        segs = [_rand_segment(rng, rng.choice([0, 1, 2, 5, 9])) for _ in range(nseg)]
        nw = _table_words(nseg) + sum(len(s) for s in segs)
        assert nw <= MSG_WORDS
        ref = _write_check(ctx, segs, ("nseg", nseg, "nch", nch))
        if nseg < 512:
            m = sp.read_message(ref, ctx=ctx)
            for a, b in zip(segs, m.segments()):
                assert np.array_equal(a, b)


def _pin_edge_words():
    """The largest one-segment message the pinned mid-size path takes:
    o_dout + bound + 16 <= kWritePinMax (capi.hip capnp_packed_write_message)."""
    def r16(x):
        return (x + 15) & ~15

    def fits(nw):
        nch = 2
        o_off = r16(nw * 8)
        o_tot = o_off + r16((nch + 1) * 8)
        o_dout = o_tot + r16((nch + 1) * 8)
        bound = 8 * nw + (nw + nch) // 2 + 2 * nch + 16
        return o_dout + bound + 16 <= PIN_MAX
    lo, hi = 1, 1 << 20
    while lo + 1 < hi:
        mid = (lo + hi) // 2
        lo, hi = (mid, hi) if fits(mid) else (lo, mid)
    return lo


def test_write_pinned_path_edge(ctx):
    """A one-segment message on each side of the pinned mid-size path's 4 MiB
    staging limit (past it the segments go through pageable copies)."""
    rng = np.random.default_rng(4)
    edge = _pin_edge_words()
    for nw in (edge - 1, edge, edge + 1):
        n = nw - 1
        w = rng.integers(0, 1 << 63, n, dtype=np.uint64)
        w[rng.random(n) < 0.3] = 0
        w[rng.random(n) < 0.05] = 0x0102030405060708  # 0xFF heads, literal runs
        _write_check(ctx, [w], ("pin edge", nw))


@pytest.mark.parametrize("k", [BODY_WORDS - 1, BODY_WORDS, BODY_WORDS + 1])
def test_read_message_body_edge(ctx, k):
    """read_message of one-segment bodies of 65535, 65536 (the first size on
    the block decode) and 65537 words: whole, with the next message's bytes
    after it, truncated by one byte, and truncated inside the body; status,
    consumed bytes and the words equal the oracle's read_message."""
    for kind in (0, 1, 2):
        w = O.gen_fill(np.array([0, k], np.uint64), kinds=np.array([kind], np.uint8),
                       pz=O.PZ30, id0=7000 + kind)
        st, msg = O.write_message([w])
        assert st == 0
        nxt = O.write_message([w[:5]])[1]
        for data in (msg, msg + nxt, msg[:-1], msg[:len(msg) // 2]):
            rst, rsegs, rused = O.read_message(bytes(data))
            r, body, used = _read_message_call(ctx.handle, data)
            assert r == rst, (k, kind, len(data), r, rst)
            if rst == 0:
                assert used == rused
                assert np.array_equal(body[:k], rsegs[0])
