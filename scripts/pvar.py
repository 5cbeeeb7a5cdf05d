#!/usr/bin/env python3
"""Times the pack kernel of several library variants, with and without the
record sync index (diagnostic; `make -C capnproto-rust_amd variant NAME=..
DEFS=..` builds build/abl/libcapnp_packed_NAME.so).

    python3 scripts/pvar.py LIB.so [LIB.so ...] [--pz N]
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
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, tile_chunks_for
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    ref, ref_off = ctx.pack_batch(words, offs)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    cap = ctx.batch_bound_bytes(n * cw, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sync = torch.empty(ctx.sync_entries(n * cw), dtype=torch.int32, device="cuda")
    tc = tile_chunks_for(n * cw, n)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    libs = []
    for path in a.libs:
        L = C.CDLL(os.path.abspath(path))
        L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
        L.capnp_ctx_create.restype = vp
        L.capnp_gpu_pack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
        L.capnp_gpu_pack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, u32, vp]
        L.capnp_ctx_reserve.argtypes = [vp, sz]
        st = C.c_int(0)
        h = vp(L.capnp_ctx_create(0, C.byref(st)))
        L.capnp_ctx_reserve(h, n)
        L.capnp_pack_tile_words.restype = u32
        libs.append((path, L, h, tile_chunks_for(n * cw, n, lib=L)))
    times = {}
    oks = {}
    # rounds interleave the libraries so clock drift hits all of them alike
    for rnd in range(a.rounds):
        for path, L, h, tc in libs:
            for use_sync in (False, True):
                for it in range(a.iters + 1):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    if use_sync:
                        r = L.capnp_gpu_pack_batch_sync_tuned(
                            h, P(words.data_ptr()), P(offs.data_ptr()), n, P(out.data_ptr()), cap,
                            P(oo.data_ptr()), P(sync.data_ptr()), tc, P(stream.cuda_stream))
                    else:
                        r = L.capnp_gpu_pack_batch_tuned(
                            h, P(words.data_ptr()), P(offs.data_ptr()), n, P(out.data_ptr()), cap,
                            P(oo.data_ptr()), tc, P(stream.cuda_stream))
                    e1.record(stream)
                    e1.synchronize()
                    assert r == 0, r
                    if it:
                        times.setdefault((path, use_sync), []).append(e0.elapsed_time(e1) * 1e3)
                ok = torch.equal(oo, ref_off) and torch.equal(out[:ref.numel()], ref)
                oks[(path, use_sync)] = oks.get((path, use_sync), True) and ok
    for path, _, _, _ in libs:
        for use_sync in (False, True):
            ts = sorted(times[(path, use_sync)])
            print(f"{os.path.basename(path)} sync={int(use_sync)}: pack {ts[0]:.1f} us "
                  f"(median {ts[len(ts) // 2]:.1f}) ok={oks[(path, use_sync)]}", flush=True)


if __name__ == "__main__":
    main()
