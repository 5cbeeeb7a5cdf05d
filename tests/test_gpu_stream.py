"""GPU parity of the streaming host batch API (capnp_stream_pack_batch /
capnp_stream_unpack_batch) against the CPU oracle.

Slices are made small so that every batch runs through many slices: both
staging slots, the slot-reuse waits and the per-slice offset rebasing are
exercised, along with a chunk larger than a slice, empty chunks and an
output buffer that is too small.
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


def _host(a, dtype, pin=True):
    t = torch.from_numpy(np.ascontiguousarray(a).view(dtype).copy())
    return t.pin_memory() if pin else t


def _stream_round_trip(ctx, words, offs, slice_words, pin=True):
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    n = len(offs) - 1
    hw = _host(words, np.int64, pin)
    ho = _host(offs, np.int64, pin)
    cap = ctx.batch_bound_bytes(int(offs[-1]), n)
    out = torch.zeros(max(cap, 1), dtype=torch.uint8)
    out = out.pin_memory() if pin else out
    oo = torch.zeros(n + 1, dtype=torch.int64)
    total = ctx.stream_pack(hw, ho, out, oo, slice_words=slice_words)
    assert total == len(ref)
    assert np.array_equal(oo.numpy().view(np.uint64), ref_offs)
    assert np.array_equal(out.numpy()[:total], ref)
    back = torch.zeros(max(len(words), 1), dtype=torch.int64)
    back = back.pin_memory() if pin else back
    status = torch.full((max(n, 1),), -1, dtype=torch.int32)
    consumed = torch.zeros(max(n, 1), dtype=torch.int64)
    ctx.stream_unpack(out, oo, ho, back, status, consumed, slice_words=slice_words)
    assert (status.numpy()[:n] == 0).all()
    assert np.array_equal(consumed.numpy()[:n].view(np.uint64), np.diff(ref_offs))
    assert np.array_equal(back.numpy()[:len(words)].view(np.uint64), words)


@pytest.mark.parametrize("slice_words", [0, 64, 1000, 4096])
def test_stream_edge_sizes(ctx, slice_words):
    sizes = [0, 1, 2, 7, 63, 64, 65, 128, 129, 255, 256, 257, 511, 513, 1000, 5000, 0, 0, 3]
    offs = np.concatenate([[0], np.cumsum(sizes * 3)]).astype(np.uint64)
    for kind in (0, 1, 2):
        words = O.gen_fill(offs, kind0=kind, pz=O.PZ30)
        _stream_round_trip(ctx, words, offs, slice_words)


def test_stream_many_slices_random(ctx):
    rng = np.random.default_rng(11)
    sizes = rng.integers(0, 700, 3000)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ80)
    _stream_round_trip(ctx, words, offs, slice_words=20000)
    _stream_round_trip(ctx, words, offs, slice_words=20000, pin=False)


def test_stream_pack_small_capacity(ctx):
    sizes = [100] * 50
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    st, ref, ref_offs = O.pack_batch(words, offs)
    cap = len(ref) // 2
    out = torch.full((cap + 64,), 0xAB, dtype=torch.uint8).pin_memory()
    oo = torch.zeros(51, dtype=torch.int64)
    from capnp_amd import _lib
    L = _lib.lib()
    import ctypes as C
    hw, ho = _host(words, np.int64), _host(offs, np.int64)
    r = L.capnp_stream_pack_batch(ctx.handle, C.c_void_p(hw.data_ptr()),
                                  C.c_void_p(ho.data_ptr()), 50,
                                  C.c_void_p(out.data_ptr()), cap, C.c_void_p(oo.data_ptr()),
                                  700)
    assert r == O.STATUS["BUFFER_NOT_LARGE_ENOUGH"]
    assert int(oo[50]) == len(ref)  # the size that was needed
    assert np.array_equal(out.numpy()[:cap], ref[:cap])
    assert (out.numpy()[cap:] == 0xAB).all()  # nothing at or past out_cap


def test_stream_unpack_errors_vs_oracle(ctx):
    rng = random.Random(23)
    chunks, lens = [], []
    for _ in range(400):
        n = rng.choice([1, 3, 40, 64, 130])
        w = np.array([rng.choice([0, 0xFF, 0x0102030405060708, rng.getrandbits(64)])
                      for _ in range(n)], np.uint64)
        st, k = O.pack(w.tobytes())
        k = bytearray(k)
        if rng.random() < 0.4 and len(k) > 1:
            k = k[:rng.randrange(len(k))]
        chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(chunks), np.uint8)
    ref_words, ref_st, ref_used = O.unpack_batch(packed, in_offs, out_offs)
    ok = ref_st == 0
    assert ok.sum() > 50 and (~ok).sum() > 50
    n = len(lens)
    words = torch.zeros(int(out_offs[-1]), dtype=torch.int64).pin_memory()
    status = torch.full((n,), -1, dtype=torch.int32)
    consumed = torch.zeros(n, dtype=torch.int64)
    hp, hi, ho = _host(packed, np.uint8), _host(in_offs, np.int64), _host(out_offs, np.int64)
    ctx.stream_unpack(hp, hi, ho, words, status, consumed, slice_words=1500)
    assert np.array_equal(status.numpy(), ref_st)
    assert np.array_equal(consumed.numpy().view(np.uint64), ref_used)  # error chunks too
    gw = words.numpy().view(np.uint64)
    for c in np.nonzero(ok)[0]:
        a, b = int(out_offs[c]), int(out_offs[c + 1])
        assert np.array_equal(gw[a:b], ref_words[a:b])


def test_stream_empty(ctx):
    out = torch.zeros(16, dtype=torch.uint8)
    oo = torch.full((1,), 7, dtype=torch.int64)
    words = torch.zeros(1, dtype=torch.int64)
    offs = torch.zeros(1, dtype=torch.int64)
    assert ctx.stream_pack(words, offs, out, oo) == 0
    assert int(oo[0]) == 0
    ctx.stream_unpack(out, oo, offs, words, torch.zeros(1, dtype=torch.int32))
