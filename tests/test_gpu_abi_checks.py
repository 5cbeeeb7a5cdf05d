"""The C ABI refuses offset arrays that would send a kernel outside the
caller's buffers: decreasing offsets (a chunk, message or slice of negative
length) and, where the buffer length is passed, an end past it.  Each call
goes through ctypes exactly as a Rust/C caller would and must return
CAPNP_E_INVALID_ARGUMENT (64) with no kernel fault; a valid call on the same
context afterwards still works.  (The reference takes slices, which cannot be
backwards or out of range: serialize.rs:53-97, serialize_packed.rs:300-304.)"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

BAD = 64


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from capnp_amd import Context, _lib
    c = Context(0)
    yield c, _lib.lib(), torch
    c.close()


def _p(t):
    return C.c_void_p(t.data_ptr())


def _dev(torch, a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a).astype(dtype)).cuda()


def _words(torch, n):
    return _dev(torch, O.gen_fill(np.array([0, n], np.uint64)).view(np.int64), np.int64)


def test_pack_batch_backwards_offsets(env):
    ctx, L, torch = env
    w = _words(torch, 512)
    out = torch.empty(8192, dtype=torch.uint8, device="cuda")
    oo = torch.empty(5, dtype=torch.int64, device="cuda")
    bad = _dev(torch, [0, 300, 100, 400, 512], np.int64)  # chunk 1 runs backwards
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.capnp_gpu_pack_batch(ctx.handle, _p(w), _p(bad), 4, _p(out), out.numel(),
                                  _p(oo), s) == BAD
    sync = torch.empty(64, dtype=torch.int32, device="cuda")
    assert L.capnp_gpu_pack_batch_sync(ctx.handle, _p(w), _p(bad), 4, _p(out), out.numel(),
                                       _p(oo), _p(sync), s) == BAD
    good = _dev(torch, [0, 100, 300, 400, 512], np.int64)
    assert L.capnp_gpu_pack_batch(ctx.handle, _p(w), _p(good), 4, _p(out), out.numel(),
                                  _p(oo), s) == 0
    torch.cuda.synchronize()
    st, ref, ref_off = O.pack_batch(w.cpu().numpy().view(np.uint64),
                                    np.array([0, 100, 300, 400, 512], np.uint64))
    assert np.array_equal(out[:len(ref)].cpu().numpy(), ref)


def test_unpack_batch_backwards_offsets(env):
    ctx, L, torch = env
    words = O.gen_fill(np.array([0, 256], np.uint64))
    st, packed, poff = O.pack_batch(words, np.array([0, 128, 256], np.uint64))
    dp = _dev(torch, packed, np.uint8)
    back = torch.empty(256, dtype=torch.int64, device="cuda")
    status = torch.empty(2, dtype=torch.int32, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    in_bad = _dev(torch, [0, int(poff[2]), int(poff[1])], np.int64)
    out_ok = _dev(torch, [0, 128, 256], np.int64)
    assert L.capnp_gpu_unpack_batch(ctx.handle, _p(dp), _p(in_bad), 2, _p(back), _p(out_ok),
                                    _p(status), None, s) == BAD
    out_bad = _dev(torch, [0, 200, 128], np.int64)
    in_ok = _dev(torch, poff.view(np.int64), np.int64)
    assert L.capnp_gpu_unpack_batch(ctx.handle, _p(dp), _p(in_ok), 2, _p(back), _p(out_bad),
                                    _p(status), None, s) == BAD
    assert L.capnp_gpu_unpack_batch_resync(ctx.handle, _p(dp), _p(in_bad), 2, _p(back),
                                           _p(out_ok), _p(status), None, s) == BAD
    assert L.capnp_gpu_unpack_batch(ctx.handle, _p(dp), _p(in_ok), 2, _p(back), _p(out_ok),
                                    _p(status), None, s) == 0
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert np.array_equal(back.cpu().numpy().view(np.uint64), words)


def test_flat_slices_checked(env):
    ctx, L, torch = env
    from capnp_amd import _lib
    msg = np.array([0, 1], np.uint32).tobytes() + b"\x07" * 8  # 1 segment of 1 word
    buf = msg * 3
    d_buf = _dev(torch, np.frombuffer(buf, np.uint8), np.uint8)
    segs = torch.empty(16, dtype=torch.int32, device="cuda")
    mso = torch.empty(4, dtype=torch.int64, device="cuda")
    status = torch.empty(3, dtype=torch.int32, device="cuda")
    o = _lib.ReaderOptionsC(8 << 20, 1, 64)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = len(buf)
    for offs in ([0, 16, 8, 48], [0, 16, 32, n + 8], [n + 16, n + 16, n + 16, n + 16]):
        d_off = _dev(torch, offs, np.int64)
        for no_alloc in (0, 1):
            assert L.capnp_gpu_read_flat_messages(
                ctx.handle, _p(d_buf), n, _p(d_off), 3, C.byref(o), no_alloc, _p(segs), 16,
                _p(mso), _p(status), None, None, s) == BAD, offs
    d_off = _dev(torch, [0, 16, 32, 48], np.int64)
    assert L.capnp_gpu_read_flat_messages(ctx.handle, _p(d_buf), n, _p(d_off), 3, C.byref(o),
                                          0, _p(segs), 16, _p(mso), _p(status), None, None,
                                          s) == 0
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()


def test_messages_checked(env):
    ctx, L, torch = env
    from capnp_amd import _lib
    st, b = O.write_message([np.arange(1, 20, dtype=np.uint64)])
    assert st == 0
    stream = b * 3
    dp = _dev(torch, np.frombuffer(stream, np.uint8), np.uint8)
    words = torch.empty(256, dtype=torch.int64, device="cuda")
    mwo = torch.empty(4, dtype=torch.int64, device="cuda")
    segs = torch.empty(16, dtype=torch.int64, device="cuda")
    mso = torch.empty(4, dtype=torch.int64, device="cuda")
    status = torch.empty(3, dtype=torch.int32, device="cuda")
    o = _lib.ReaderOptionsC(8 << 20, 1, 64)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    bad = _dev(torch, [0, 2 * len(b), len(b), 3 * len(b)], np.int64)
    assert L.capnp_gpu_read_messages(ctx.handle, _p(dp), _p(bad), 3, C.byref(o), 0, _p(words),
                                     256, _p(mwo), _p(segs), 16, _p(mso), _p(status), None,
                                     s) == BAD
    good = _dev(torch, [0, len(b), 2 * len(b), 3 * len(b)], np.int64)
    assert L.capnp_gpu_read_messages(ctx.handle, _p(dp), _p(good), 3, C.byref(o), 0, _p(words),
                                     256, _p(mwo), _p(segs), 16, _p(mso), _p(status), None,
                                     s) == 0
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    # write_messages: message segment offsets past total_segs, and backwards
    w = _dev(torch, np.arange(1, 31, dtype=np.uint64).view(np.int64), np.int64)
    swo = _dev(torch, [0, 10, 20, 30], np.int64)
    out = torch.empty(1024, dtype=torch.uint8, device="cuda")
    mbo = torch.empty(3, dtype=torch.int64, device="cuda")
    for mseg in ([0, 2, 5], [0, 2, 1]):
        dm = _dev(torch, mseg, np.int64)
        assert L.capnp_gpu_write_messages(ctx.handle, _p(w), _p(swo), _p(dm), 2, 3, 30, _p(out),
                                          out.numel(), _p(mbo), s) == BAD, mseg
    swo_bad = _dev(torch, [0, 20, 10, 30], np.int64)
    dm = _dev(torch, [0, 1, 3], np.int64)
    assert L.capnp_gpu_write_messages(ctx.handle, _p(w), _p(swo_bad), _p(dm), 2, 3, 30, _p(out),
                                      out.numel(), _p(mbo), s) == BAD
    # segment offsets past the words d_words holds (total_words): rejected
    # before any segment is read
    swo_past = _dev(torch, [0, 10, 20, 4000], np.int64)
    assert L.capnp_gpu_write_messages(ctx.handle, _p(w), _p(swo_past), _p(dm), 2, 3, 30,
                                      _p(out), out.numel(), _p(mbo), s) == BAD
    assert L.capnp_gpu_write_messages(ctx.handle, _p(w), _p(swo), _p(dm), 2, 3, 29, _p(out),
                                      out.numel(), _p(mbo), s) == BAD
    assert L.capnp_gpu_write_messages(ctx.handle, _p(w), _p(swo), _p(dm), 2, 3, 30, _p(out),
                                      out.numel(), _p(mbo), s) == 0
    torch.cuda.synchronize()


def test_long_chunk_paths_checked(env):
    """The long-chunk paths (mean chunk >= 512 words: word-tile pack, and the
    block decode without the index, which the batch entry point hands its
    already-checked ranges to) refuse backwards offsets too, and decode a
    valid batch afterwards."""
    ctx, L, torch = env
    n_words = 4096
    w = _words(torch, n_words)
    host = w.cpu().numpy().view(np.uint64)
    offs = np.array([0, 1500, 2600, n_words], np.uint64)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = torch.empty(n_words * 10 + 64, dtype=torch.uint8, device="cuda")
    oo = torch.empty(4, dtype=torch.int64, device="cuda")
    bad = _dev(torch, [0, 2600, 1500, n_words], np.int64)
    assert L.capnp_gpu_pack_batch(ctx.handle, _p(w), _p(bad), 3, _p(out), out.numel(),
                                  _p(oo), s) == BAD
    good = _dev(torch, offs.view(np.int64), np.int64)
    assert L.capnp_gpu_pack_batch(ctx.handle, _p(w), _p(good), 3, _p(out), out.numel(),
                                  _p(oo), s) == 0
    torch.cuda.synchronize()
    st, ref, ref_off = O.pack_batch(host, offs)
    assert np.array_equal(oo.cpu().numpy().view(np.uint64), ref_off)
    assert np.array_equal(out[:len(ref)].cpu().numpy(), ref)
    back = torch.zeros(n_words, dtype=torch.int64, device="cuda")
    status = torch.empty(3, dtype=torch.int32, device="cuda")
    in_ok = _dev(torch, ref_off.view(np.int64), np.int64)
    in_bad = _dev(torch, [0, int(ref_off[2]), int(ref_off[1]), int(ref_off[3])], np.int64)
    out_bad = _dev(torch, [0, 2600, 1500, n_words], np.int64)
    for fn in (L.capnp_gpu_unpack_batch, L.capnp_gpu_unpack_batch_resync):
        assert fn(ctx.handle, _p(out), _p(in_bad), 3, _p(back), _p(good), _p(status), None,
                  s) == BAD
        assert fn(ctx.handle, _p(out), _p(in_ok), 3, _p(back), _p(out_bad), _p(status), None,
                  s) == BAD
    assert L.capnp_gpu_unpack_batch(ctx.handle, _p(out), _p(in_ok), 3, _p(back), _p(good),
                                    _p(status), None, s) == 0
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert np.array_equal(back.cpu().numpy().view(np.uint64), host)
