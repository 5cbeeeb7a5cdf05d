"""Termination and fallback of the index-free decode (csrc/resync.hip) on
streams where the speculative chains never couple: in a literal-run region
(serialize_packed.rs:394-433 packs incompressible words as 0xFF records of
255 raw words) only the true chain settles a tile, so the tiles hand their
exits on one by one (look-back) and each needs several rounds.  The tests
cap the rounds per tile through capnp_resync_max_passes (the hook's name
predates the look-back) to reach the fallbacks.  The decode must still
terminate and return the reference's bytes:

* capnp_gpu_unpack_batch_resync fails the capped tiles' chunks, which its
  block decode then walks serially, each as one unit (serial = 3);
* the stream reader's whole-record cut (capnp_resync_decode_prefix, reads
  of 64 KiB and more) falls back to an exact serial walk for the cut.

The oracle (oracle/packed_oracle.c, restating serialize_packed.rs:80-228 and
:304-439) gives the packed stream and checks the decode.  Also the round-3
hang inputs (literal and zero runs across blocks and tiles, read through
large reads and the batch resync) once more."""
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


def _literal_words(n, seed):
    # every byte non-zero: a stream of 0xFF records, each with 255 raw words
    rng = np.random.default_rng(seed)
    return rng.integers(1 << 56, 1 << 63, n, dtype=np.uint64) | np.uint64(0x0101010101010101)


@pytest.fixture
def pass_cap():
    """Rounds per tile capped at 1 (capnp_resync_max_passes), restored after."""
    from capnp_amd import _lib
    old = _lib.lib().capnp_resync_max_passes(1)
    yield
    _lib.lib().capnp_resync_max_passes(old)


def test_resync_batch_literal_region_past_pass_cap(ctx, pass_cap):
    n = (4 << 20) // 8  # 4 MiB of literal words: ~160 tiles, each past the round cap
    w = _literal_words(n, 3)
    st, p = O.pack(w.tobytes())
    assert st == 0
    packed = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).cuda()
    in_off = torch.tensor([0, len(p)], dtype=torch.int64, device="cuda")
    out_off = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    words = torch.zeros(n, dtype=torch.int64, device="cuda")
    status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    consumed = torch.zeros(1, dtype=torch.int64, device="cuda")
    passes, serial = ctx.unpack_batch_resync_into(packed, in_off, out_off, words, status,
                                                  consumed)
    assert serial == 3 and passes >= 1, (passes, serial)
    assert int(status[0]) == 0 and int(consumed[0]) == len(p)
    assert np.array_equal(words.cpu().numpy().view(np.uint64), w)


def test_reader_large_read_literal_region_past_pass_cap(ctx, pass_cap):
    """Large reads of a 4 MiB literal stream with the rounds capped: the
    reader's whole-record cut (capnp_resync_decode_prefix) does not converge
    and takes the serial cut, with the same bytes (the reader
    used to fail with CAPNP_E_HIP there)."""
    from capnp_amd import serialize_packed_async as A
    n = (4 << 20) // 8
    w = _literal_words(n, 4)
    u = w.tobytes()
    st, p = O.pack(u)
    assert st == 0

    class Plain:
        def __init__(self, data):
            self.data, self.pos = bytes(data), 0

        def read(self, k):
            b = self.data[self.pos:self.pos + k]
            self.pos += len(b)
            return b

    for size in (8 << 20, (1 << 20) + 8):
        pr = A.PackedRead(Plain(p))
        got = bytearray()
        while True:
            b = pr.read(size)
            if not b:
                break
            assert 0 < len(b) <= size
            got += b
        assert bytes(got) == u, size


def test_literal_region_converges_uncapped(ctx):
    """A 20 MiB literal region with the default cap: the fix passes carry the
    true chain through all ~800 tiles (tiles later in a pass read exits their
    predecessors wrote in that pass) and the block decode is exact."""
    n = (20 << 20) // 8
    w = _literal_words(n, 5)
    st, p = O.pack(w.tobytes())
    assert st == 0
    packed = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).cuda()
    in_off = torch.tensor([0, len(p)], dtype=torch.int64, device="cuda")
    out_off = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    words = torch.zeros(n, dtype=torch.int64, device="cuda")
    status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    passes, serial = ctx.unpack_batch_resync_into(packed, in_off, out_off, words, status)
    assert serial == 0 and passes < 512, (passes, serial)
    assert int(status[0]) == 0
    assert np.array_equal(words.cpu().numpy().view(np.uint64), w)


def test_resync_hang_inputs_repeat(ctx):
    """The round-3 hang inputs (test_batch_long_runs' chunks, _mixed_words'
    stream), each decoded several times (round 3's fix passes raced on the
    predecessor's exit; the look-back reads it once per workgroup)."""
    chunks = []
    for n in (255, 256, 257, 300, 511, 512, 513, 1023, 1500):
        for lead in (0, 1, 63):
            z = np.zeros(n + lead, np.uint64)
            z[:lead] = 0x0102030400000000
            chunks.append(z)
            lit = np.full(n + lead, 0x1112131415161718, np.uint64)
            lit[:lead] = 0x0000000400000001
            chunks.append(lit)
            mix = np.full(n + lead, 0x11121314151617, np.uint64)
            mix[lead] = 0x1112131415161718
            chunks.append(mix)
    offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).astype(np.uint64)
    words = np.concatenate(chunks)
    st, packed, poffs = O.pack_batch(words, offs)
    assert st == 0
    dp = torch.from_numpy(np.asarray(packed).copy()).cuda()
    di = torch.from_numpy(poffs.view(np.int64).copy()).cuda()
    do = torch.from_numpy(offs.view(np.int64).copy()).cuda()
    for _ in range(5):
        out = torch.zeros(len(words), dtype=torch.int64, device="cuda")
        status = torch.full((len(chunks),), -1, dtype=torch.int32, device="cuda")
        ctx.unpack_batch_resync_into(dp, di, do, out, status)
        assert (status.cpu().numpy() == 0).all()
        assert np.array_equal(out.cpu().numpy().view(np.uint64), words)


def test_lookback_ticket_reset_at_whole_tile_bound(ctx):
    """A unit whose block bound (packed bytes / 512 + chunks + 1) is a whole
    number of 64-block tiles, decoded twice on one context: k_tile's ticket
    sits in the record array's last word and must be zeroed before every
    launch (a stale ticket would hand every tile an index past the batch)."""
    n = 4000  # 0xFF records: 32032 packed bytes -> 62 + 2 = 64 blocks
    w = _literal_words(n, 6)
    st, p = O.pack(w.tobytes())
    assert st == 0 and len(p) // 512 + 2 == 64, len(p)
    packed = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).cuda()
    in_off = torch.tensor([0, len(p)], dtype=torch.int64, device="cuda")
    out_off = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    for _ in range(3):
        words = torch.zeros(n, dtype=torch.int64, device="cuda")
        status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
        passes, serial = ctx.unpack_batch_resync_into(packed, in_off, out_off, words, status)
        assert serial == 0 and int(status[0]) == 0, (passes, serial, int(status[0]))
        assert np.array_equal(words.cpu().numpy().view(np.uint64), w)
