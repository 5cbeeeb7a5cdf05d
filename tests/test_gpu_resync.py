"""GPU parity of the index-free decode (capnp_gpu_unpack_batch_resync,
SURVEY §8f row 2) against the CPU oracle's read_exact (oracle/packed_oracle.c,
which restates serialize_packed.rs:80-228 + io.rs:16-31).

The resync decode walks each chunk's tag chain block by block from
speculative starts, so the cases that matter are the ones where a
speculative start lands badly: literal runs that span several blocks, zero
runs, chunks shorter than one block, one chunk many blocks long, and
malformed chunks (decoded serially, each on its own, and coming out with the
oracle's statuses while the rest of the batch keeps the block decode)."""
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
    c = Context(0)
    yield c
    c.close()


def dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint8:
        return torch.from_numpy(a.copy()).cuda() if len(a) else torch.zeros(8, dtype=torch.uint8,
                                                                            device="cuda")
    return torch.from_numpy(a.view(np.int64).copy()).cuda()


def resync(ctx, packed, in_offs, out_offs):
    n = len(in_offs) - 1
    nw = max(int(out_offs[-1]), 1)
    words = torch.zeros(nw, dtype=torch.int64, device="cuda")
    status = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
    consumed = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    passes, serial = ctx.unpack_batch_resync_into(dev(packed), dev(in_offs), dev(out_offs),
                                                  words, status, consumed)
    return (words.cpu().numpy().view(np.uint64)[:int(out_offs[-1])], status.cpu().numpy()[:n],
            consumed.cpu().numpy().view(np.uint64)[:n], passes, serial)


def packed_batch(sizes, kinds, pz=O.PZ30, id0=0):
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kinds=np.asarray(kinds, np.uint8), pz=pz, id0=id0)
    st, packed, poffs = O.pack_batch(words, offs)
    assert st == 0
    return words, offs, packed, poffs


@pytest.mark.parametrize("seed", [0, 1])
def test_resync_mixed_sizes(ctx, seed):
    """Config-4 shape: log-uniform 8..8192-word chunks, 80 % iid / 10 % long
    zero runs / 10 % long literal runs; bit-exact, no serial fallback."""
    rng = np.random.default_rng(seed)
    n = 600
    sizes = np.exp(rng.uniform(np.log(8), np.log(8192), n)).astype(np.uint64)
    kinds = rng.choice([0, 1, 2], n, p=[0.8, 0.1, 0.1])
    words, offs, packed, poffs = packed_batch(sizes, kinds, id0=1000 * seed)
    g, st, used, passes, serial = resync(ctx, packed, poffs, offs)
    assert serial == 0 and passes >= 1
    assert (st == 0).all()
    assert np.array_equal(used, np.diff(poffs))
    assert np.array_equal(g, words)


@pytest.mark.parametrize("kind,pz", [(0, O.PZ30), (0, O.PZ80), (1, 0), (2, 0)])
def test_resync_one_long_chunk(ctx, kind, pz):
    """A single read unit hundreds of blocks long (a whole message body as
    read_message reads it): zero runs and literal runs spanning blocks."""
    words, offs, packed, poffs = packed_batch([1 << 18], [kind], pz=pz, id0=5 + kind)
    g, st, used, passes, serial = resync(ctx, packed, poffs, offs)
    ref, rst, rused = O.unpack_batch(packed, poffs, offs)
    assert serial == 0
    assert st[0] == rst[0] == 0 and used[0] == rused[0] == len(packed)
    assert np.array_equal(g, words)


def test_resync_literal_text(ctx):
    """100 000 'A' bytes (the overflow_test.rs:65-79 shape): literal runs of
    255 words, each record 2050 bytes, four blocks and more per record."""
    data = b"A" * 100000
    w = np.frombuffer(data, np.uint64)
    st, k = O.pack(w.tobytes())
    poffs = np.array([0, len(k)], np.uint64)
    offs = np.array([0, len(w)], np.uint64)
    g, st, used, passes, serial = resync(ctx, np.frombuffer(k, np.uint8), poffs, offs)
    assert serial == 0 and st[0] == 0 and used[0] == len(k)
    assert np.array_equal(g, w)


def test_resync_edges(ctx):
    """Empty chunks, 1-word chunks, chunks of exactly one block, zero-word
    output with packed bytes present (read() of an empty buffer reads
    nothing), all in one batch."""
    sizes = [0, 1, 0, 2, 64, 0, 1, 300, 5000, 0]
    kinds = [0, 0, 0, 1, 2, 0, 2, 1, 0, 0]
    words, offs, packed, poffs = packed_batch(sizes, kinds, id0=9)
    g, st, used, passes, serial = resync(ctx, packed, poffs, offs)
    ref, rst, rused = O.unpack_batch(packed, poffs, offs)
    assert serial == 0
    assert np.array_equal(st, rst) and np.array_equal(used, rused)
    assert np.array_equal(g, words)


def _rand_chunk(rng, n):
    w = np.zeros(n, np.uint64)
    b = w.view(np.uint8)
    style = rng.random()
    for i in range(n):
        r = rng.random()
        if style < 0.3:
            if r < 0.1:
                b[8 * i:8 * i + 8] = [rng.randrange(256) for _ in range(8)]
        elif style < 0.6:
            vals = [rng.randrange(1, 256) for _ in range(8)]
            if r < 0.05:
                vals[rng.randrange(8)] = 0
            b[8 * i:8 * i + 8] = vals
        else:
            b[8 * i:8 * i + 8] = [rng.randrange(256) if rng.random() < 0.5 else 0
                                  for _ in range(8)]
    return w


def test_resync_malformed_chunks_alone_serial(ctx):
    """Truncated, corrupted, mis-sized, over-long and byte-less chunks:
    statuses, consumed counts and the good chunks' words equal the oracle's;
    only the failing chunks leave the block decode (serial == 3), and the
    whole output, partial words of failing chunks included, equals the serial
    batch unpack's (capnp_gpu_unpack_batch)."""
    rng = random.Random(23)
    chunks, lens = [], []
    for _ in range(300):
        n = rng.choice([1, 7, 64, 130, 700, 2000])
        st, k = O.pack(_rand_chunk(rng, n).tobytes())
        k = bytearray(k)
        r = rng.random()
        if r < 0.02:
            k = bytearray()  # no packed bytes for n > 0 words
        elif r < 0.15 and len(k) > 1:
            k = k[:rng.randrange(len(k))]
        elif r < 0.3 and len(k):
            k[rng.randrange(len(k))] = rng.choice([0, 0xFF, rng.randrange(256)])
        elif r < 0.4:
            n = max(0, n + rng.choice([-3, -1, 1, 4]))
        elif r < 0.45:
            k += bytes([0x01, 0x07])  # spare bytes after a complete unit
        chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(chunks), np.uint8)
    ref, rst, rused = O.unpack_batch(packed, in_offs, out_offs)
    g, st, used, passes, serial = resync(ctx, packed, in_offs, out_offs)
    assert serial == 3
    assert np.array_equal(st, rst)
    sw = torch.zeros(max(int(out_offs[-1]), 1), dtype=torch.int64, device="cuda")
    sst = torch.empty(len(chunks), dtype=torch.int32, device="cuda")
    ctx.unpack_batch_into(dev(packed), dev(in_offs), dev(out_offs), sw, sst)
    assert np.array_equal(sst.cpu().numpy(), rst)
    assert np.array_equal(g, sw.cpu().numpy().view(np.uint64)[:len(g)])
    ok = rst == 0
    assert ok.sum() > 50 and (~ok).sum() > 50
    assert np.array_equal(used, rused)  # error chunks too
    for c in np.nonzero(ok)[0]:
        a, b = int(out_offs[c]), int(out_offs[c + 1])
        assert np.array_equal(g[a:b], ref[a:b]), c
    # the same batch without a consumed array (d_consumed = NULL)
    w2 = torch.zeros(max(int(out_offs[-1]), 1), dtype=torch.int64, device="cuda")
    st2 = torch.full((len(chunks),), -1, dtype=torch.int32, device="cuda")
    passes2, serial2 = ctx.unpack_batch_resync_into(dev(packed), dev(in_offs), dev(out_offs),
                                                    w2, st2)
    assert serial2 == 3
    assert np.array_equal(st2.cpu().numpy(), rst)
    assert np.array_equal(w2.cpu().numpy().view(np.uint64)[:len(g)], g)


def test_resync_config4_round_trip(ctx):
    """~128 MiB of config-4 chunks packed on the GPU and decoded index-free:
    round trip identical to the input and to the serial unpack's output."""
    rng = np.random.default_rng(44)
    sizes = np.exp(rng.uniform(np.log(8), np.log(8192), 16384)).astype(np.int64)
    kinds = rng.choice([0, 1, 2], len(sizes), p=[0.8, 0.1, 0.1]).astype(np.uint8)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(sizes)])).cuda()
    words = torch.empty(int(offs[-1]), dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=O.PZ30, kinds=torch.from_numpy(kinds).cuda(), id0=3)
    packed, poffs = ctx.pack_batch(words, offs)
    n = len(sizes)
    back = torch.zeros_like(words)
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    passes, serial = ctx.unpack_batch_resync_into(packed, poffs, offs, back, st)
    assert serial == 0
    assert (st == 0).all().item()
    assert torch.equal(back, words)


def test_resync_short_chunks_dispatch(ctx):
    """Batches of short chunks (config-2 shape) go straight to the batch
    unpack; results are the same either way."""
    words, offs, packed, poffs = packed_batch([128] * 2000, [0] * 2000, id0=31)
    g, st, used, passes, serial = resync(ctx, packed, poffs, offs)
    assert serial == 2 and passes == 0
    assert (st == 0).all() and np.array_equal(used, np.diff(poffs))
    assert np.array_equal(g, words)


def test_resync_two_streams_one_ctx(ctx):
    """Two index-free decodes queued back to back on different streams of one
    context (the second call must not reset the shared workspace under the
    first one's kernels: it waits for them by an event)."""
    w1, o1, p1, po1 = packed_batch([1 << 16] * 4, [0, 1, 0, 2], id0=77)
    w2, o2, p2, po2 = packed_batch([1 << 15] * 6, [1, 0, 2, 0, 0, 0], pz=O.PZ80, id0=78)
    args = []
    for (w, o, p, po) in ((w1, o1, p1, po1), (w2, o2, p2, po2)):
        n = len(o) - 1
        args.append((dev(p), dev(po), dev(o), torch.zeros(int(o[-1]), dtype=torch.int64, device="cuda"),
                     torch.full((n,), -1, dtype=torch.int32, device="cuda"),
                     torch.zeros(n, dtype=torch.int64, device="cuda")))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(3):
        for a in args:
            a[3].zero_()
        torch.cuda.synchronize()
        ctx.unpack_batch_resync_into(*args[0], stream=s1.cuda_stream, stats=False)
        ctx.unpack_batch_resync_into(*args[1], stream=s2.cuda_stream, stats=False)
        torch.cuda.synchronize()
        for (w, o, p, po), a in zip(((w1, o1, p1, po1), (w2, o2, p2, po2)), args):
            assert (a[4].cpu().numpy() == 0).all(), rep
            assert np.array_equal(a[5].cpu().numpy().view(np.uint64), np.diff(po)), rep
            assert np.array_equal(a[3].cpu().numpy().view(np.uint64), w), rep
