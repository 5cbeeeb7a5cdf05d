"""Config 1 on the GPU: the carsales request stream (BASELINE.json configs[0];
SURVEY.md §8d) generated on the device, packed and unpacked by the gfx950
kernels, against the CPU oracle (oracle/carsales_oracle.c + packed_oracle.c).

  * the device generator equals the oracle's stream word for word (1 GiB);
  * 1 Mi x 1 KiB carsales-shaped segments (the north_star workload: the
    request stream cut into 128-word chunks) pack byte for byte like the
    oracle, over the whole batch, and unpack back, with and without the
    record sync index;
  * whole request messages through capnp_gpu_write_messages /
    capnp_gpu_read_messages equal the oracle's write_message / read_message
    (the reference benchmark's `bytes reuse packed` codec calls,
    benchmark.rs:235-241)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, CW = 1 << 20, 128  # 1 Mi x 1 KiB


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def stream(ctx):
    words = torch.empty(N * CW, dtype=torch.int64, device="cuda")
    offs = ctx.gen_carsales(words)
    torch.cuda.synchronize()
    ref, roffs, _ = O.carsales_stream(N * CW)
    return words, offs, ref, roffs


def test_generator_matches_oracle(stream):
    words, offs, ref, roffs = stream
    assert np.array_equal(offs, roffs)
    got = words.cpu().numpy().view(np.uint64)
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, f"first mismatch at word {bad[:4]}"


def test_generator_skip(ctx):
    words = torch.empty(50_000, dtype=torch.int64, device="cuda")
    offs = ctx.gen_carsales(words, skip_requests=1000)
    ref, roffs, _ = O.carsales_stream(50_000, skip=1000)
    assert np.array_equal(offs, roffs)
    assert np.array_equal(words.cpu().numpy().view(np.uint64), ref)


@pytest.mark.parametrize("sync", [False, True])
def test_carsales_chunks_pack_unpack_full(ctx, stream, sync):
    """The north_star workload, whole batch byte for byte vs the oracle."""
    from capnp_amd import tile_chunks_for, unpack_tile_chunks_for
    words, _, ref, _ = stream
    offs = torch.arange(0, (N + 1) * CW, CW, dtype=torch.int64, device="cuda")
    cap = ctx.batch_bound_bytes(N * CW, N)
    packed = torch.empty(cap, dtype=torch.uint8, device="cuda")
    poffs = torch.empty(N + 1, dtype=torch.int64, device="cuda")
    sidx = torch.empty(ctx.sync_entries(N * CW), dtype=torch.int32, device="cuda") \
        if sync else None
    ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tile_chunks_for(N * CW, N),
                        sync=sidx)
    back = torch.empty_like(words)
    status = torch.empty(N, dtype=torch.int32, device="cuda")
    consumed = torch.empty(N, dtype=torch.int64, device="cuda")
    ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed,
                          chunks_per_tile=unpack_tile_chunks_for(N * CW, N, sync=sync),
                          sync=sidx)
    torch.cuda.synchronize()
    hoffs = np.arange(0, (N + 1) * CW, CW, dtype=np.uint64)
    st, rpk, rpo = O.pack_batch(ref, hoffs, threads=16)
    assert st == 0
    assert np.array_equal(poffs.cpu().numpy().view(np.uint64), rpo)
    P = int(rpo[-1])
    assert 0.6 < P / (8 * N * CW) < 0.8  # carsales packs to ~0.70
    assert np.array_equal(packed[:P].cpu().numpy(), rpk)
    assert int((status != 0).sum()) == 0
    assert torch.equal(back, words)
    assert torch.equal(consumed, poffs[1:] - poffs[:-1])
    if sync:
        rs = O.sync_index(rpk, rpo, hoffs)
        got = sidx.cpu().numpy().view(np.uint32)
        given = got != 0xFFFFFFFF
        assert given.mean() > 0.99 and np.array_equal(got[given], rs[given])


def test_carsales_messages_write_read(ctx):
    """Whole request messages (one segment each, ~12 KB) through the batch
    message framing, against the oracle's write_message / read_message."""
    nmsg = 2000
    st = O.carsales_seed()
    segs = [O.carsales_request(st)[0] for _ in range(nmsg)]
    seg_off = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.int64)
    msg_seg_off = np.arange(nmsg + 1, dtype=np.int64)
    words = np.concatenate(segs)
    d_words = torch.from_numpy(words.view(np.int64).copy()).cuda()
    packed, mo = ctx.write_messages(d_words, torch.from_numpy(seg_off).cuda(),
                                    torch.from_numpy(msg_seg_off).cuda())
    got = packed.cpu().numpy().tobytes()
    mo_h = mo.cpu().numpy()
    pos = 0
    for i, s in enumerate(segs):
        r, ref = O.write_message([s])
        assert r == 0 and mo_h[i] == pos and got[pos:pos + len(ref)] == ref, i
        pos += len(ref)
    assert pos == len(got)
    w, mwo, sg, mso, stt, cons = ctx.read_messages(packed, mo, len(words) + 16, nmsg + 16)
    torch.cuda.synchronize()
    assert int((stt != 0).sum()) == 0
    assert torch.equal(cons, mo[1:] - mo[:-1])
    assert np.array_equal(mwo.cpu().numpy(), seg_off)
    assert torch.equal(w[:len(words)], d_words)
    assert np.array_equal(sg[:nmsg].cpu().numpy(), np.diff(seg_off))
