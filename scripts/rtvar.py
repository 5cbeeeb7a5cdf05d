#!/usr/bin/env python3
"""Times pack + unpack (both with the record sync index) of several whole-
library variants on the config-2 batch, interleaved over rounds, and checks
the round trip (diagnostic; `make -C capnproto-rust_amd fvariant NAME=..
DEFS=..` builds build/abl/libcapnp_packed_f_NAME.so).  Each library packs its
own index, so variants may differ in the index format.

    python3 scripts/rtvar.py LIB.so [LIB.so ...] [--pz N] [--rounds R]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    cap = ctx.batch_bound_bytes(n * cw, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    tc = tile_chunks_for(n * cw, n)
    libs = []
    for path in a.libs:
        L = C.CDLL(os.path.abspath(path))
        L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
        L.capnp_ctx_create.restype = vp
        L.capnp_ctx_reserve.argtypes = [vp, sz]
        L.capnp_sync_index_entries.argtypes = [sz]
        L.capnp_sync_index_entries.restype = sz
        L.capnp_gpu_pack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, u32, vp]
        L.capnp_gpu_unpack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, u32,
                                                        vp]
        L.capnp_unpack_tile_words.restype = u32
        L.capnp_unpack_sync_tile_words.restype = u32
        st = C.c_int(0)
        h = vp(L.capnp_ctx_create(0, C.byref(st)))
        L.capnp_ctx_reserve(h, n)
        sync = torch.empty(int(L.capnp_sync_index_entries(n * cw)), dtype=torch.int32,
                           device="cuda")
        utc = unpack_tile_chunks_for(n * cw, n, lib=L, sync=True)
        L.capnp_pack_tile_words.restype = u32
        libs.append((path, L, h, sync, utc, tile_chunks_for(n * cw, n, lib=L)))
    tp, tu, oks = {}, {}, {}

    def timed(fn):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r = fn()
        e1.record(stream)
        e1.synchronize()
        assert r == 0, r
        return e0.elapsed_time(e1) * 1e3

    for rnd in range(a.rounds):
        for path, L, h, sync, utc, tc in libs:
            for it in range(a.iters + 1):
                t = timed(lambda: L.capnp_gpu_pack_batch_sync_tuned(
                    h, P(words.data_ptr()), P(offs.data_ptr()), n, P(out.data_ptr()), cap,
                    P(oo.data_ptr()), P(sync.data_ptr()), tc, P(stream.cuda_stream)))
                if it:
                    tp.setdefault(path, []).append(t)
            for it in range(a.iters + 1):
                t = timed(lambda: L.capnp_gpu_unpack_batch_sync_tuned(
                    h, P(out.data_ptr()), P(oo.data_ptr()), n, P(back.data_ptr()),
                    P(offs.data_ptr()), P(sync.data_ptr()), P(status.data_ptr()), None, utc,
                    P(stream.cuda_stream)))
                if it:
                    tu.setdefault(path, []).append(t)
            ok = torch.equal(back, words) and int((status != 0).sum()) == 0
            oks[path] = oks.get(path, True) and ok
            back.zero_()
    for path, _, _, _, utc, _ in libs:
        p, u = sorted(tp[path]), sorted(tu[path])
        print(f"{os.path.basename(path)}: pack {p[0]:.1f} (med {p[len(p) // 2]:.1f}) "
              f"unpack {u[0]:.1f} (med {u[len(u) // 2]:.1f}) sum {p[0] + u[0]:.1f} us "
              f"utc={utc} ok={oks[path]}", flush=True)


if __name__ == "__main__":
    main()
