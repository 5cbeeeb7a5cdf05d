#!/usr/bin/env python3
"""Phase breakdown of the unpack kernel from the UNPACK_PROF=1 build
(`make -C capnproto-rust_amd variant FILE=unpack NAME=uprof DEFS=-DUNPACK_PROF=1`): s_memtime cycles of wave 0 per phase
(stage bytes, walk, expand) summed over staged tiles.  Diagnostic only.

    python3 scripts/unpack_prof.py [--chunks N] [--chunk-words W] [--utc T]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--utc", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--lib", default="")
    ap.add_argument("--sync", action="store_true", help="the indexed path (record sync index)")
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, unpack_tile_chunks_for
    L = C.CDLL(a.lib or os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_uprof.so"))
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
    L.capnp_ctx_create.restype = vp
    L.capnp_gpu_unpack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, u32, vp]
    L.capnp_gpu_unpack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, u32, vp]
    L.capnp_unpack_prof.argtypes = [vp, C.c_int]
    st = C.c_int(0)
    h = vp(L.capnp_ctx_create(0, C.byref(st)))
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    sync = None
    if a.sync:
        cap = ctx.batch_bound_bytes(n * cw, n)
        packed = torch.empty(cap, dtype=torch.uint8, device="cuda")
        poffs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        sync = torch.empty(ctx.sync_entries(n * cw), dtype=torch.int32, device="cuda")
        ctx.pack_batch_into(words, offs, packed, poffs, sync=sync)
    else:
        packed, poffs = ctx.pack_batch(words, offs)
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    utc = a.utc or unpack_tile_chunks_for(n * cw, n, sync=a.sync)
    buf = (C.c_ulonglong * 16)()
    ntiles = (n + utc - 1) // utc
    trace = torch.zeros(ntiles * 8, dtype=torch.int64, device="cuda")
    L.capnp_unpack_trace.argtypes = [vp]
    L.capnp_unpack_trace(C.c_void_p(trace.data_ptr()))
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    for it in range(a.iters + 1):
        torch.cuda.synchronize()
        L.capnp_unpack_prof(buf, 1)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if sync is not None:
            L.capnp_gpu_unpack_batch_sync_tuned(h, P(packed.data_ptr()), P(poffs.data_ptr()), n,
                                                P(back.data_ptr()), P(offs.data_ptr()),
                                                P(sync.data_ptr()), P(status.data_ptr()), None,
                                                utc, P(stream.cuda_stream))
        else:
            L.capnp_gpu_unpack_batch_tuned(h, P(packed.data_ptr()), P(poffs.data_ptr()), n,
                                           P(back.data_ptr()), P(offs.data_ptr()),
                                           P(status.data_ptr()), None, utc, P(stream.cuda_stream))
        e1.record(stream)
        e1.synchronize()
        L.capnp_unpack_prof(buf, 1)
        if it == 0:
            continue
        ok = torch.equal(back, words)
        T = trace.view(ntiles, 8).cpu().numpy().astype("int64")
        st = T[:, 4] == 0
        d = lambda a, b: (T[st, b] - T[st, a]).mean() / 100.0
        life = (T[st, 3] - T[st, 0]) / 100.0
        span = (T[st, 3].max() - T[st, 0].min()) / 100.0
        print(f"iter {it}: {e0.elapsed_time(e1) * 1e3:.1f} us ok={ok} staged={st.sum()} "
              f"exact-walk chunks={buf[0]} "
              f"global={(~st).sum()} per tile: stage={d(0, 1):.2f}us walk={d(1, 2):.2f}us "
              f"expand={d(2, 3):.2f}us life={life.mean():.2f}us "
              f"concurrency={life.sum() / max(span, 1e-9):.0f} "
              + (f"phaseB-iters={T[st, 5].mean():.2f} walk_segment={T[st, 6].mean():.0f}cyc "
                 f"phaseA={T[st, 7].mean():.0f}cyc" if a.sync else
                 f"| wave 0: spec={d(1, 5):.2f}us rounds={d(5, 6):.2f}us desc={d(6, 7):.2f}us "
                 f"status+barrier={d(7, 2):.2f}us"))

if __name__ == "__main__":
    main()
