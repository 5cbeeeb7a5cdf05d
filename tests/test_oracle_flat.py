"""Oracle for unpacked flat-slice framing, pinned by the
reference's own tests:
  serialize.rs:1063-1093  read_message_from_flat_slice_with_remainder
  serialize.rs:1095-1115  read_message_from_flat_slice_too_short
  serialize.rs:1045-1060  test_round_trip_slice_segments (quickcheck property)
  no_alloc_buffer_segments.rs:505-519  ..._message_postfix
  no_alloc_buffer_segments.rs:521-544  ..._message_invalid
and cross-checked against an independent pure-Python restatement of
serialize.rs:53-78 / :448-510 and no_alloc_buffer_segments.rs:22-92.
"""
import random
import struct

import numpy as np

import oracle_lib as O

OK, FILL, NSEG, TOO_LARGE, ENDS, EMPTY, NOT_ALIGNED = 0, 4, 6, 8, 12, 13, 14


def flat_message(segments):
    """serialize::flatten_segments / write_segment_table layout
    (serialize.rs:546-560, :595-664): segments are lists of bytes."""
    n = len(segments)
    t = struct.pack("<I", n - 1) + b"".join(struct.pack("<I", len(s) // 8) for s in segments)
    if len(t) % 8:
        t += b"\0" * 4
    return t + b"".join(bytes(s) for s in segments)


def aligned(data, pad=0):
    """An 8-byte aligned np.uint8 copy of `data` starting at byte `pad`."""
    w = np.zeros((len(data) + pad + 15) // 8, np.uint64)
    b = w.view(np.uint8)
    b[pad:pad + len(data)] = np.frombuffer(bytes(data), np.uint8)
    return b


def py_flat(data, no_alloc, limit=O.DEFAULT_TRAVERSAL_LIMIT, align=0):
    """Independent restatement -> (status, lens, table_bytes, consumed); on
    MessageEndsPrematurely the last two are its (header, body) payload."""
    n = len(data)
    u32 = lambda p: struct.unpack_from("<I", data, p)[0]
    if not no_alloc:
        if n == 0:
            return EMPTY, [], 0, 0
        if n < 8:
            return FILL, [], 0, 0
        cnt = (u32(0) + 1) & 0xFFFFFFFF
        if cnt >= 512 or cnt == 0:
            return NSEG, [], 0, 0
        lens = [u32(4)]
        pos = 8
        if cnt > 1:
            rest = 8 if cnt < 4 else (cnt & ~1) * 4
            if n - pos < rest:
                return FILL, [], 0, 0
            lens += [u32(pos + 4 * i) for i in range(cnt - 1)]
            pos += rest
        if limit is not None and sum(lens) > limit:
            return TOO_LARGE, [], 0, 0
        if sum(lens) > (n - pos) // 8:
            return ENDS, [], sum(lens), (n - pos) // 8
    else:
        if align % 8:
            return NOT_ALIGNED, [], 0, 0
        if n < 4:
            return ENDS, [], 4, n
        cnt = u32(0) + 1
        if cnt >= 512:
            return NSEG, [], 0, 0
        pos, lens = 4, []
        for _ in range(cnt):
            if n - pos < 4:
                return ENDS, [], 4, n - pos
            lens.append(u32(pos))
            pos += 4
        if limit is not None and sum(lens) > limit:
            return TOO_LARGE, [], 0, 0
        if cnt % 2 == 0:
            if n - pos < 4:
                return ENDS, [], 4, n - pos
            pos += 4
        if n - pos < 8 * sum(lens):
            return ENDS, [], sum(lens), (n - pos) // 8
    return OK, lens, pos, pos + 8 * sum(lens)


def oracle(data, no_alloc, limit=O.DEFAULT_TRAVERSAL_LIMIT, pad=0):
    return O.read_flat_message(aligned(data, pad), pad, len(data), no_alloc, limit)


def test_with_remainder():
    segs = [[123, 0, 0, 0, 0, 0, 0, 0], [4, 0, 0, 0, 0, 0, 0, 0, 5, 0, 0, 0, 0, 0, 0, 0]]
    extra = bytes([9, 9, 9, 9, 9, 9, 9, 9, 8, 7, 6, 5, 4, 3, 2, 1])
    data = flat_message(segs) + extra
    for na in (False, True):
        st, lens, tb, used = oracle(data, na)
        assert st == OK and lens == [1, 2] and tb == 16
        assert data[used:] == extra


def test_too_short():
    data = flat_message([[1, 0, 0, 0, 0, 0, 0, 0], [2, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 0, 0, 0, 0]])
    for na in (False, True):
        for k in range(len(data)):
            assert oracle(data[:k], na)[0] != OK
    assert oracle(b"", False)[0] == EMPTY
    assert oracle(b"", True)[0] == ENDS


def test_no_alloc_postfix_and_invalid():
    data = flat_message([[1, 2, 3, 4, 5, 6, 7, 8]]) + bytes([11, 12, 13, 14, 15, 16, 0, 0])
    st, lens, tb, used = oracle(data, True)
    assert st == OK and data[used:] == bytes([11, 12, 13, 14, 15, 16, 0, 0])
    assert oracle(bytes([0, 2, 0, 0]) + bytes(513 * 8), True)[0] == NSEG
    assert oracle(bytes([0, 0, 0, 0]), True)[0] == ENDS
    assert oracle(bytes([0, 0, 0, 0, 0, 0, 0]), True)[0] == ENDS
    assert oracle(bytes([255, 255, 255, 255]), True)[0] == NSEG
    assert oracle(bytes([255, 255, 255, 255]) + bytes(8), False)[0] == NSEG


def test_alignment_and_limit():
    data = flat_message([bytes(16)])
    assert oracle(data, True, pad=4)[0] == NOT_ALIGNED
    assert oracle(data, False, pad=4)[0] == OK  # the alloc path checks no alignment
    assert oracle(data, False, limit=1)[0] == TOO_LARGE
    assert oracle(data, True, limit=1)[0] == TOO_LARGE
    assert oracle(data, True, limit=None)[0] == OK


def test_round_trip_property_and_restatement():
    rng = random.Random(7)
    for it in range(3000):
        nseg = rng.choice([1, 1, 2, 3, 4, 5, 6, rng.randrange(1, 520)])
        segs = [bytes(rng.randrange(256) for _ in range(8 * rng.randrange(0, 3)))
                for _ in range(nseg)]
        data = bytearray(flat_message(segs) + bytes(rng.randrange(0, 24)))
        mode = rng.random()
        if mode < 0.3:
            data = data[:rng.randrange(0, len(data) + 1)]
        elif mode < 0.5 and data:
            data[rng.randrange(min(len(data), 24))] = rng.randrange(256)
        data = bytes(data)
        pad = rng.choice([0, 0, 0, 4])
        limit = rng.choice([O.DEFAULT_TRAVERSAL_LIMIT, None, 3])
        for na in (False, True):
            got = oracle(data, na, limit, pad)
            assert got == py_flat(data, na, limit, pad), (it, na)
            if got[0] == OK and mode >= 0.5:
                assert got[1] == [len(s) // 8 for s in segs]


def test_message_ends_prematurely_payload():
    """capnp/tests/buffer_size_too_small.rs:5-20: one segment claiming 2 words
    over 1 word of body is MessageEndsPrematurely(2, 1); the no-alloc reader
    reads the same bytes as a 1-segment table of length 2 (u32 count 0, u32
    length 2) and reports the same pair (no_alloc_buffer_segments.rs:77-80)."""
    data = bytes([0, 0, 0, 0, 2, 0, 0, 0]) + bytes(8)
    for na in (False, True):
        assert oracle(data, na) == (ENDS, [], 2, 1)
    assert oracle(bytes(3), True) == (ENDS, [], 4, 3)  # read_u32_le :254-257
