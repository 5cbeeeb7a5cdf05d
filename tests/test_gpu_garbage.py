"""Arbitrary bytes through the GPU decoders, against the C oracle:
  * quickcheck test_unpack (capnp/src/serialize_packed.rs:584-593): any
    byte string through read_exact must not crash; here every status,
    consumed count and the words of every OK chunk must equal the oracle's,
    in one batch, with and without a (garbage) record sync index;
  * the fuzz target capnp/fuzz/fuzzers/serialize_packed_read_no_alloc.rs:5-13
    (read_message_no_alloc into a 512-word buffer, traversal limit 256) on
    random and mutated streams: status, table and body bytes, consumed.
The corpus is seeded (no fuzzer engine is available offline)."""
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


def _garbage(rng, n):
    alphabet = [0, 0, 0xFF, 0xFF, 1, 2, 0x81, 0xF0, 0x0F]
    return bytes(rng.choice(alphabet) if rng.random() < 0.5 else rng.randrange(256)
                 for _ in range(n))


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def test_unpack_random_bytes_vs_oracle(ctx):
    import torch
    rng = random.Random(2024)
    chunks, lens = [], []
    for _ in range(4000):
        n = rng.choice([0, 1, 2, 3, 9, 10, 11, 17, 40, 100, 300])
        d = _garbage(rng, n)
        chunks.append(d)
        # test_unpack reads len * 8 bytes; also shorter and empty outputs
        lens.append(rng.choice([n, n, max(0, n // 3), 0, 1, 2]))
    in_offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(chunks), np.uint8)
    ref_w, ref_st, ref_used = O.unpack_batch(packed, in_offs, out_offs)
    ok = ref_st == 0
    assert ok.sum() > 300 and (~ok).sum() > 300
    pk = torch.from_numpy(packed.copy()).cuda()
    for utc in (0, 1, 7, 64):
        words, status, consumed = ctx.unpack_batch(pk, _dev(in_offs), _dev(out_offs),
                                                   chunks_per_tile=utc)
        torch.cuda.synchronize()
        assert np.array_equal(status.cpu().numpy(), ref_st), utc
        assert np.array_equal(consumed.cpu().numpy().view(np.uint64), ref_used), utc
        gw = words.cpu().numpy().view(np.uint64)
        for c in np.nonzero(ok)[0]:
            a, b = int(out_offs[c]), int(out_offs[c + 1])
            assert np.array_equal(gw[a:b], ref_w[a:b]), (utc, c)
    # a garbage record sync index changes nothing (it is never trusted)
    total = int(out_offs[-1])
    sync = torch.from_numpy(np.frombuffer(rng.randbytes(4 * ctx.sync_entries(total)),
                                          np.int32).copy()).cuda()
    n = len(chunks)
    back = torch.zeros(max(total, 1), dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    cons = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(pk, _dev(in_offs), _dev(out_offs), back, st, cons, sync=sync)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), ref_st)
    assert np.array_equal(cons.cpu().numpy().view(np.uint64), ref_used)


def _mutations(rng):
    segs = [np.array([rng.getrandbits(64) if rng.random() < 0.6 else 0
                      for _ in range(rng.choice([0, 1, 3, 20, 200]))], np.uint64)
            for _ in range(rng.choice([1, 1, 2, 4, 9]))]
    st, b = O.write_message(segs)
    b = bytearray(b)
    for _ in range(rng.choice([0, 1, 1, 2, 5])):
        if b:
            b[rng.randrange(len(b))] = rng.choice([0, 0xFF, rng.randrange(256)])
    if rng.random() < 0.3 and b:
        b = b[:rng.randrange(len(b))]
    return bytes(b)


def test_fuzz_read_message_no_alloc_vs_oracle(ctx):
    from capnp_amd import serialize_packed as sp, CapnpError
    rng = random.Random(77)
    opts = sp.ReaderOptions(traversal_limit_in_words=256)
    seen = set()
    for i in range(1500):
        data = _garbage(rng, rng.choice([0, 1, 7, 8, 9, 16, 30, 80, 400])) if i % 2 else \
            _mutations(rng)
        buf = np.zeros(512, np.uint64)
        ref = O.read_message_no_alloc(data, 512, limit=256)
        try:
            m = sp.read_message_no_alloc(sp.SliceRead(data), buf, opts, ctx=ctx)
            st = 0
        except CapnpError as e:
            st = e.status
        seen.add(st)
        assert st == ref[0], (i, data[:40], st, ref[0])
        if st == 0:
            nseg, tb, bb = ref[2], ref[3], ref[4]
            assert len(m) == nseg
            assert np.array_equal(buf.view(np.uint8)[:tb + bb], ref[1][:tb + bb]), i
    assert len(seen) >= 5, seen  # OK and several error kinds were exercised
