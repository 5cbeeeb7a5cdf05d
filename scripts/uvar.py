#!/usr/bin/env python3
"""Times the unpack kernel of several library variants on one packed batch
(diagnostic; `make -C capnproto-rust_amd uvariant NAME=.. DEFS=..`).  For
variants built with -DUNPACK_PROF=1 it also prints the per-tile phase means.

    python3 scripts/uvar.py LIB.so [LIB.so ...] [--pz N] [--chunk-words W]
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
    ap.add_argument("--utc", type=int, default=0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--sync", action="store_true", help="unpack through the record sync index")
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, unpack_tile_chunks_for
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    packed, poffs = ctx.pack_batch(words, offs)
    sync = None
    if a.sync:
        sync = torch.empty(ctx.sync_entries(n * cw), dtype=torch.int32, device="cuda")
        po2 = torch.empty_like(poffs)
        buf = torch.empty(ctx.batch_bound_bytes(n * cw, n), dtype=torch.uint8, device="cuda")
        ctx.pack_batch_into(words, offs, buf, po2, sync=sync)
        packed, poffs = buf, po2
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    for path in a.libs:
        L = C.CDLL(os.path.abspath(path))
        vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
        L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
        L.capnp_ctx_create.restype = vp
        L.capnp_gpu_unpack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, u32, vp]
        if sync is not None:
            L.capnp_gpu_unpack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp,
                                                            u32, vp]
        L.capnp_unpack_tile_words.restype = u32
        L.capnp_unpack_sync_tile_words.restype = u32
        st = C.c_int(0)
        h = vp(L.capnp_ctx_create(0, C.byref(st)))
        utc = a.utc or unpack_tile_chunks_for(n * cw, n, lib=L, sync=a.sync)
        ntiles = (n + utc - 1) // utc
        prof = hasattr(L, "capnp_unpack_trace")
        trace = None
        if prof:
            trace = torch.zeros(ntiles * 8, dtype=torch.int64, device="cuda")
            L.capnp_unpack_trace.argtypes = [vp]
            L.capnp_unpack_trace(P(trace.data_ptr()))
        back = torch.empty_like(words)
        status = torch.empty(n, dtype=torch.int32, device="cuda")
        ts = []
        for it in range(a.iters + 1):
            back.zero_()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if sync is None:
                r = L.capnp_gpu_unpack_batch_tuned(h, P(packed.data_ptr()), P(poffs.data_ptr()),
                                                   n, P(back.data_ptr()), P(offs.data_ptr()),
                                                   P(status.data_ptr()), None, utc,
                                                   P(stream.cuda_stream))
            else:
                r = L.capnp_gpu_unpack_batch_sync_tuned(
                    h, P(packed.data_ptr()), P(poffs.data_ptr()), n, P(back.data_ptr()),
                    P(offs.data_ptr()), P(sync.data_ptr()), P(status.data_ptr()), None, utc,
                    P(stream.cuda_stream))
            e1.record(stream)
            e1.synchronize()
            assert r == 0, r
            if it:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ok = torch.equal(back, words) and int((status != 0).sum()) == 0
        line = f"{os.path.basename(path)}: utc={utc} unpack {min(ts):.1f} us (mean {sum(ts)/len(ts):.1f}) ok={ok}"
        if prof:
            T = trace.view(ntiles, 8).cpu().numpy().astype("int64")
            s = T[:, 4] == 0
            d = lambda x, y: (T[s, y] - T[s, x]).mean() / 100.0
            life = (T[s, 3] - T[s, 0]) / 100.0
            span = (T[s, 3].max() - T[s, 0].min()) / 100.0
            if T[s, 5].max() > 0:
                line += (f" | seg loop: {T[s, 5].mean():.1f} iters, {T[s, 6].mean():.0f} cyc "
                         f"({T[s, 6].mean() / max(T[s, 5].mean(), 1):.0f}/iter)")
            line += (f" | stage {d(0, 1):.2f} walk {d(1, 2):.2f} expand {d(2, 3):.2f} us"
                     f" life {life.mean():.2f} conc {life.sum() / max(span, 1e-9):.0f}")
        if prof and hasattr(L, "capnp_unpack_prof"):
            buf = (C.c_ulonglong * 8)()
            L.capnp_unpack_prof.argtypes = [vp, C.c_int]
            L.capnp_unpack_prof(buf, 1)
            line += f" | prof {list(buf)[:4]}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
