"""GPU parity of the device batch message framing (capnp_gpu_write_messages,
SURVEY §8f row 1): every message of the batch must be byte-identical to the
oracle's serialize_packed::write_message (oracle/packed_oracle.c, pinned by
the reference's golden vectors), the message offsets must be the running
sum of their sizes, and every message must read back (oracle read_message).
"""
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
    return Context(0)


def _segment(rng, n):
    w = np.zeros(n, np.uint64)
    b = w.view(np.uint8)
    mode = rng.random()
    for i in range(n):
        r = rng.random()
        if mode < 0.3:
            if r < 0.1:
                b[8 * i:8 * i + 8] = [rng.randrange(256) for _ in range(8)]
        elif mode < 0.6:
            vals = [rng.randrange(1, 256) for _ in range(8)]
            if r < 0.2:
                vals[rng.randrange(8)] = 0
            b[8 * i:8 * i + 8] = vals
        elif r > 0.3:
            b[8 * i:8 * i + 8] = [rng.randrange(256) if rng.random() < 0.56 else 0
                                  for _ in range(8)]
    return w


def _check_messages(ctx, msgs):
    seg_lens = [len(s) for m in msgs for s in m]
    seg_off = np.concatenate([[0], np.cumsum(seg_lens)]).astype(np.int64)
    msg_seg_off = np.concatenate([[0], np.cumsum([len(m) for m in msgs])]).astype(np.int64)
    words = (np.concatenate([s for m in msgs for s in m]) if seg_off[-1] else
             np.zeros(1, np.uint64))
    dw = torch.from_numpy(words.view(np.int64).copy()).cuda()
    packed, mo = ctx.write_messages(dw, torch.from_numpy(seg_off).cuda(),
                                    torch.from_numpy(msg_seg_off).cuda())
    torch.cuda.synchronize()
    got = packed.cpu().numpy().tobytes()
    mo = mo.cpu().numpy()
    pos = 0
    for i, m in enumerate(msgs):
        st, ref = O.write_message(m)
        assert st == 0
        assert mo[i] == pos, i
        assert got[pos:pos + len(ref)] == ref, (i, [len(s) for s in m])
        st2, segs, used = O.read_message(got[pos:pos + len(ref)], limit=None,
                                         body_cap=sum(len(s) for s in m) + 16)
        assert st2 == 0 and used == len(ref)
        assert len(segs) == len(m) and all(np.array_equal(a, b) for a, b in zip(segs, m))
        pos += len(ref)
    assert mo[-1] == pos == len(got)


def test_write_messages_random(ctx):
    rng = random.Random(7)
    msgs = []
    for _ in range(300):
        nseg = rng.choice([1, 1, 2, 3, 4, 5, 8, 17])
        msgs.append([_segment(rng, rng.choice([0, 1, 2, 63, 64, 65, 128, 300]))
                     for _ in range(nseg)])
    _check_messages(ctx, msgs)


def test_write_messages_edges(ctx):
    rng = random.Random(3)
    msgs = [
        [np.zeros(0, np.uint64)],                        # one empty segment
        [np.zeros(300, np.uint64)],                      # one long zero run
        [np.full(600, 0x0102030405060708, np.uint64)],   # literal run > 255
        [np.zeros(0, np.uint64)] * 6,                     # empty segments only
        [_segment(rng, 5) for _ in range(511)],          # the most segments a reader takes
        [_segment(rng, 1000)],
    ]
    _check_messages(ctx, msgs)
    _check_messages(ctx, msgs[:1])


def test_write_messages_carsales_like_batch(ctx):
    # many single-segment 1 KiB messages (the config-2 shape) plus a few
    # multi-segment ones
    rng = random.Random(9)
    msgs = [[_segment(rng, 128)] for _ in range(2000)]
    for k in range(0, 2000, 97):
        msgs[k] = [_segment(rng, 60), _segment(rng, 68)]
    _check_messages(ctx, msgs)


def test_write_messages_region_overflow(ctx):
    """Segments that pack to 8.5 bytes per word (a 0xFF word, then a 6-byte
    word) overflow the pack kernel's staged regions, on the gap path that
    leaves each message's segment table in front of its bytes: those tiles'
    bytes come from the overflow pass and must still equal the oracle's."""
    rng = random.Random(21)
    adv = np.zeros(128, np.uint64)
    adv[0::2] = 0x1112131415161718
    adv[1::2] = 0x0000212223242526
    msgs = []
    for i in range(400):
        if i % 3:
            msgs.append([adv.copy() for _ in range(rng.choice([1, 2, 3]))])
        else:
            msgs.append([_segment(rng, rng.choice([0, 64, 128, 200]))])
    _check_messages(ctx, msgs)


def test_write_messages_staging_path(ctx):
    """Message offsets that do not span the batch (a segment before the first
    message and one after the last) take the staging path; the messages must
    still match the oracle byte for byte."""
    rng = random.Random(13)
    msgs = [[_segment(rng, rng.choice([0, 3, 64, 200])) for _ in range(rng.choice([1, 2, 3]))]
            for _ in range(50)]
    segs = [_segment(rng, 7)] + [s for m in msgs for s in m] + [_segment(rng, 9)]
    seg_off = np.concatenate([[0], np.cumsum([len(x) for x in segs])]).astype(np.int64)
    msg_seg_off = (1 + np.concatenate([[0], np.cumsum([len(m) for m in msgs])])).astype(np.int64)
    words = np.concatenate(segs)
    packed, mo = ctx.write_messages(torch.from_numpy(words.view(np.int64).copy()).cuda(),
                                    torch.from_numpy(seg_off).cuda(),
                                    torch.from_numpy(msg_seg_off).cuda())
    got = packed.cpu().numpy().tobytes()
    mo = mo.cpu().numpy()
    base = mo[0]
    for i, m in enumerate(msgs):
        ref = O.write_message(m)[1]
        assert got[mo[i]:mo[i + 1]] == ref, i
    assert mo[-1] - base == sum(len(O.write_message(m)[1]) for m in msgs)


# ------------------------------------------------------------ batch read side
def _read_back(ctx, packed_bytes, msg_off, words_cap, segs_cap, try_mode=False,
               limit=8 * 1024 * 1024):
    pk = torch.from_numpy(np.frombuffer(packed_bytes, np.uint8).copy()).cuda() \
        if len(packed_bytes) else torch.zeros(1, dtype=torch.uint8, device="cuda")
    mo = torch.from_numpy(np.asarray(msg_off, np.int64)).cuda()
    w, mwo, sg, mso, st, cons = ctx.read_messages(pk, mo, words_cap, segs_cap,
                                                  try_mode=try_mode, limit=limit)
    torch.cuda.synchronize()
    return (w.cpu().numpy().view(np.uint64), mwo.cpu().numpy(), sg.cpu().numpy(),
            mso.cpu().numpy(), st.cpu().numpy(), cons.cpu().numpy())


def _oracle_read(buf, try_mode, limit):
    cap = 8 * len(buf) * 32 + 64  # (zero runs expand 2040x at most per 2 bytes)
    return O.read_message(buf, try_mode=try_mode, limit=limit, body_cap=cap)


def test_read_messages_round_trip(ctx):
    rng = random.Random(21)
    msgs = []
    for _ in range(400):
        nseg = rng.choice([1, 1, 2, 3, 4, 7, 33])
        msgs.append([_segment(rng, rng.choice([0, 1, 5, 64, 65, 129, 300]))
                     for _ in range(nseg)])
    seg_lens = [len(s) for m in msgs for s in m]
    seg_off = np.concatenate([[0], np.cumsum(seg_lens)]).astype(np.int64)
    msg_seg_off = np.concatenate([[0], np.cumsum([len(m) for m in msgs])]).astype(np.int64)
    words = np.concatenate([s for m in msgs for s in m])
    packed, mo = ctx.write_messages(torch.from_numpy(words.view(np.int64).copy()).cuda(),
                                    torch.from_numpy(seg_off).cuda(),
                                    torch.from_numpy(msg_seg_off).cuda())
    w, mwo, sg, mso, st, cons = ctx.read_messages(packed, mo, len(words), len(seg_lens))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(cons.cpu().numpy(), np.diff(mo.cpu().numpy()))
    assert np.array_equal(mso.cpu().numpy(), msg_seg_off)
    assert np.array_equal(sg.cpu().numpy()[:len(seg_lens)], seg_lens)
    assert np.array_equal(mwo.cpu().numpy(), [0] + list(np.cumsum([sum(len(s) for s in m)
                                                                   for m in msgs])))
    assert np.array_equal(w.cpu().numpy().view(np.uint64)[:len(words)], words)


def test_read_messages_errors_vs_oracle(ctx):
    """Truncated, corrupted and empty messages, segment counts >= 512, the
    traversal limit: status, consumed bytes and (for OK messages) the
    segments must equal the oracle's read_message on each message alone."""
    rng = random.Random(5)
    bufs = []
    for i in range(300):
        m = [_segment(rng, rng.choice([0, 2, 40, 130])) for _ in range(rng.choice([1, 2, 5]))]
        st, b = O.write_message(m)
        b = bytearray(b)
        r = rng.random()
        if r < 0.2 and len(b) > 1:
            b = b[:rng.randrange(len(b))]                     # truncated
        elif r < 0.35 and len(b) > 2:
            b[rng.randrange(len(b))] = rng.choice([0, 0xFF, rng.randrange(256)])  # corrupted
        elif r < 0.4:
            b = bytearray()                                    # empty
        bufs.append(bytes(b))
    # a table claiming 600 segments, and one over the traversal limit
    bufs.append(bytes([0x0F, 0x57, 0x02, 0x00, 0x00, 0x00]))
    big = [np.full(100, 1, np.uint64)]
    bufs.append(O.write_message(big)[1])
    msg_off = np.concatenate([[0], np.cumsum([len(b) for b in bufs])]).astype(np.int64)
    allb = b"".join(bufs)
    for try_mode, limit in ((False, 8 * 1024 * 1024), (True, 8 * 1024 * 1024), (False, 64),
                            (True, None)):
        ref = [_oracle_read(b, try_mode, limit) for b in bufs]
        tw = sum(sum(len(s) for s in r[1]) for r in ref if r[0] == 0) + 1000000
        w, mwo, sg, mso, st, cons = _read_back(ctx, allb, msg_off, tw, 100000, try_mode, limit)
        for i, (rst, rsegs, rused) in enumerate(ref):
            assert st[i] == rst, (i, try_mode, limit, st[i], rst)
            if rst == 0:
                assert cons[i] == rused, i
                lens = sg[mso[i]:mso[i + 1]]
                assert list(lens) == [len(s) for s in rsegs], i
                body = w[mwo[i]:mwo[i + 1]]
                assert np.array_equal(body, np.concatenate(rsegs) if rsegs else body[:0]), i
