"""GPU parity of unpacked flat-slice framing (capnp_gpu_read_flat_messages,
SURVEY §8f row 4) against the oracle's read_message_from_flat_slice /
NoAllocSliceSegments::from_slice (oracle/packed_oracle.c, pinned by
tests/test_oracle_flat.py): per message the status, segment lengths, body
offset and consumed bytes must be identical, in both modes and under every
traversal limit, on batches mixing valid, truncated, corrupted, empty,
unaligned and over-limit slices.
"""
import random

import numpy as np
import pytest

import oracle_lib as O
from test_oracle_flat import flat_message

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    return Context(0)


def _batch(rng, nmsg):
    parts, offs, pos = [], [0], 0
    for _ in range(nmsg):
        nseg = rng.choice([1, 1, 1, 2, 3, 4, 7, rng.randrange(1, 520)])
        segs = [bytes(8 * rng.randrange(0, 4)) for _ in range(nseg)]
        data = bytearray(flat_message(segs) + bytes(rng.choice([0, 0, 4, 8, 16])))
        r = rng.random()
        if r < 0.15:
            data = data[:rng.randrange(0, len(data) + 1)]
        elif r < 0.25 and data:
            data[rng.randrange(min(len(data), 16))] = rng.randrange(256)
        elif r < 0.28:
            data = bytearray(rng.randrange(256) for _ in range(rng.randrange(0, 12)))
        data += bytes(-len(data) % 8)  # slices start 8-byte aligned ...
        parts.append(bytes(data))
        pos += len(data)
        offs.append(pos)
    for m in range(1, nmsg):  # ... except ~10 %, shifted by 4 (the no_alloc alignment check)
        if rng.random() < 0.1 and offs[m] + 4 <= offs[m + 1]:
            offs[m] += 4
    buf = np.zeros((pos + 15) // 8, np.uint64).view(np.uint8)
    buf[:pos] = np.frombuffer(b"".join(parts), np.uint8)
    return buf, np.array(offs, np.int64)


@pytest.mark.parametrize("no_alloc", [False, True])
@pytest.mark.parametrize("limit", [O.DEFAULT_TRAVERSAL_LIMIT, None, 2])
def test_flat_batch_matches_oracle(ctx, no_alloc, limit):
    rng = random.Random(11 + int(no_alloc) + (0 if limit is None else limit % 97))
    nmsg = 4000
    buf, offs = _batch(rng, nmsg)
    d_buf = torch.from_numpy(buf.copy()).cuda()
    d_off = torch.from_numpy(offs).cuda()
    segs, mso, st, body, used = ctx.read_flat_messages(d_buf, d_off, segs_cap=nmsg * 520,
                                                       no_alloc=no_alloc, limit=limit)
    torch.cuda.synchronize()
    segs, mso, st = segs.cpu().numpy(), mso.cpu().numpy(), st.cpu().numpy()
    body, used = body.cpu().numpy(), used.cpu().numpy()
    n_ok = 0
    for m in range(nmsg):
        a, b = int(offs[m]), int(offs[m + 1])
        est, elens, etb, eused = O.read_flat_message(buf, a, b - a, no_alloc, limit)
        assert st[m] == est, (m, st[m], est)
        got = [int(x) for x in segs[mso[m]:mso[m + 1]]]
        assert got == elens, m
        if est == 0:
            n_ok += 1
            assert body[m] == a + etb and used[m] == eused, m
        elif est == 12:  # MessageEndsPrematurely(header, body) payload
            assert (body[m], used[m]) == (etb, eused), m
        else:
            assert used[m] == 0, m
    assert n_ok > nmsg // (50 if limit == 2 else 10)  # the batch is not all errors
    assert mso[nmsg] == sum(len(O.read_flat_message(buf, int(offs[m]), int(offs[m + 1] - offs[m]),
                                                    no_alloc, limit)[1]) for m in range(nmsg))


def test_flat_empty_batch_and_small_cap(ctx):
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    segs, mso, st, body, used = ctx.read_flat_messages(buf, off, segs_cap=0)
    assert int(mso[0]) == 0 and st.numel() == 0
    data = np.zeros(16, np.uint64).view(np.uint8)
    data[:40] = np.frombuffer(flat_message([bytes(8)] * 3), np.uint8)
    d = torch.from_numpy(data.copy()).cuda()
    off = torch.tensor([0, 40], dtype=torch.int64, device="cuda")
    segs, mso, st, body, used = ctx.read_flat_messages(d, off, segs_cap=3)
    assert int(st[0]) == 0 and segs[:3].tolist() == [1, 1, 1] and int(used[0]) == 40
    from capnp_amd import CapnpError
    with pytest.raises(CapnpError):
        ctx.read_flat_messages(d, off, segs_cap=2)


def test_flat_write_messages_layout_round_trip(ctx):
    """Flat messages back to back (the layout serialize::write_message
    produces), each slice exactly one message: every message validates and
    the consumed bytes walk the stream message by message."""
    rng = np.random.default_rng(5)
    nmsg = 20000
    lens = rng.integers(0, 64, nmsg)
    nsegs = rng.integers(1, 5, nmsg)
    parts = []
    for m in range(nmsg):
        segl = [int(lens[m])] + [int(x) for x in rng.integers(0, 3, nsegs[m] - 1)]
        parts.append(flat_message([bytes(8 * l) for l in segl]))
    starts = np.cumsum([0] + [len(p) for p in parts]).astype(np.int64)
    buf = np.frombuffer(b"".join(parts), np.uint8)
    d_buf = torch.from_numpy(buf.copy()).cuda()
    d_off = torch.from_numpy(starts).cuda()
    segs, mso, st, body, used = ctx.read_flat_messages(d_buf, d_off, segs_cap=5 * nmsg,
                                                       no_alloc=True)
    st, used = st.cpu().numpy(), used.cpu().numpy()
    assert (st == 0).all()
    assert (used == np.diff(starts)).all()
    assert int(mso[-1]) == int(nsegs.sum())
    assert (body.cpu().numpy() == starts[:-1] + 8 * (nsegs // 2 + 1)).all()


def test_host_mirror_reference_cases(ctx):
    """The reference's flat-slice tests through the host mirror
    (capnp_amd.serialize): serialize.rs:1063-1115 and
    no_alloc_buffer_segments.rs:505-544."""
    from capnp_amd import CapnpError
    from capnp_amd import serialize as S
    segs = [[123, 0, 0, 0, 0, 0, 0, 0], [4, 0, 0, 0, 0, 0, 0, 0, 5, 0, 0, 0, 0, 0, 0, 0]]
    extra = bytes([9, 9, 9, 9, 9, 9, 9, 9, 8, 7, 6, 5, 4, 3, 2, 1])
    data = flat_message(segs) + extra
    dev = torch.tensor(list(data), dtype=torch.uint8, device="cuda")
    for fn in (S.read_message_from_flat_slice, S.read_message_from_flat_slice_no_alloc):
        got, rest = fn(dev)
        assert [g.cpu().tolist() for g in got] == segs
        assert bytes(rest.cpu().tolist()) == extra
    short = flat_message([[1, 0, 0, 0, 0, 0, 0, 0], [2, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 0, 0, 0, 0]])
    dshort = torch.tensor(list(short), dtype=torch.uint8, device="cuda")
    for k in range(len(short)):
        for fn in (S.read_message_from_flat_slice, S.read_message_from_flat_slice_no_alloc):
            with pytest.raises(CapnpError):
                fn(dshort[:k])
    with pytest.raises(CapnpError) as e:
        S.read_message_from_flat_slice(dshort[:0])
    assert e.value.kind == "EmptySlice"
    bad = torch.tensor([255, 255, 255, 255], dtype=torch.uint8, device="cuda")
    with pytest.raises(CapnpError) as e:
        S.read_message_from_flat_slice_no_alloc(bad)
    assert e.value.kind == "InvalidNumberOfSegments"


def test_serialize_batch_two_phase_cap_and_checks(ctx):
    """The public batch entry point sizes the segment array exactly (no
    511-per-message default): 200k one-segment messages need 200k entries.
    Bad slice offsets, strided tensors and short caps raise instead of
    reading out of bounds."""
    from capnp_amd import CapnpError
    from capnp_amd import serialize as S
    nmsg = 200_000
    one = np.frombuffer(flat_message([bytes(8)] * 3), np.uint8)  # 3 segments, 40 bytes
    buf = torch.from_numpy(np.tile(one, nmsg).copy()).cuda()
    off = torch.arange(nmsg + 1, dtype=torch.int64, device="cuda") * one.size
    segs, mso, st, body, used = S.read_flat_messages(buf, off)
    assert segs.numel() == 3 * nmsg and int(mso[-1]) == 3 * nmsg
    assert bool((st == 0).all()) and bool((used == one.size).all())
    for bad in ([0, 40, 20], [0, 40, 10**9], [-8, 40]):
        with pytest.raises(CapnpError):
            S.read_flat_messages(buf, torch.tensor(bad, dtype=torch.int64, device="cuda"))
    with pytest.raises(CapnpError):
        S.read_flat_messages(buf[::2], off[:2])
    with pytest.raises(CapnpError):
        S.read_message_from_flat_slice(buf[::2])


def test_message_ends_prematurely_payload(ctx):
    """capnp/tests/buffer_size_too_small.rs: one segment claiming 2 words with
    1 word of body is MessageEndsPrematurely(2, 1); the pair comes back in
    body_off / consumed."""
    data = np.array([0, 0, 0, 0, 2, 0, 0, 0] + [0] * 8, np.uint8)
    d = torch.from_numpy(data).cuda()
    off = torch.tensor([0, 16], dtype=torch.int64, device="cuda")
    segs, mso, st, body, used = ctx.read_flat_messages(d, off)
    assert (int(st[0]), int(body[0]), int(used[0])) == (12, 2, 1)
