#!/usr/bin/env python3
"""Phase breakdown of the pack kernel from the PACK_PROF=1 build
(`make -C capnproto-rust_amd prof`): s_memtime cycles per phase summed over
workgroups (wave 0), look-back spin rounds and fallbacks.  Diagnostic only.

    python3 scripts/pack_prof.py [--chunks N] [--chunk-words W] [--tc T]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))

PHASES = ["advance+meta", "compute", "bar1", "publish+plan", "bar2", "lookback",
          "bar_fin", "copy_out", "bar_end", "pre_finish"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--tc", type=int, default=0)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, tile_chunks_for
    path = os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_prof.so")
    L = C.CDLL(path)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
    L.capnp_ctx_create.restype = vp
    L.capnp_gpu_pack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
    L.capnp_ctx_reserve.argtypes = [vp, sz]
    L.capnp_pack_prof.argtypes = [vp, C.c_int]
    st = C.c_int(0)
    h = vp(L.capnp_ctx_create(0, C.byref(st)))
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    ref_out, ref_oo = ctx.pack_batch(words, offs)
    cap = ctx.batch_bound_bytes(n * cw, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    tc = a.tc or tile_chunks_for(n * cw, n)
    L.capnp_ctx_reserve(h, n)
    buf = (C.c_ulonglong * 16)()
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    for it in range(a.iters + 1):
        torch.cuda.synchronize()
        L.capnp_pack_prof(buf, 1)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        L.capnp_gpu_pack_batch_tuned(h, P(words.data_ptr()), P(offs.data_ptr()), n,
                                     P(out.data_ptr()), cap, P(oo.data_ptr()), tc,
                                     P(stream.cuda_stream))
        e1.record(stream)
        e1.synchronize()
        L.capnp_pack_prof(buf, 1)
        if it == 0:
            continue
        ok = torch.equal(oo, ref_oo) and torch.equal(out[:ref_out.numel()], ref_out)
        wgs = max(buf[15], 1)
        tot = sum(buf[i] for i in range(10))
        print(f"iter {it}: {e0.elapsed_time(e1) * 1e3:.1f} us, ok={ok}, WGs={buf[15]}, "
              f"tiles={buf[14]}, spins={buf[12]}, fallbacks={buf[13]}, "
              f"cycles/WG={tot / wgs:.0f}")
        print("   " + "  ".join(f"{PHASES[i]}={100 * buf[i] / max(tot, 1):.1f}%"
                                 for i in range(10)))


if __name__ == "__main__":
    main()
