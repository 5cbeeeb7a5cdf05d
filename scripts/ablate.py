#!/usr/bin/env python3
"""Interleaved A/B timing of diagnostic library variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Variants are built by
`make -C capnproto-rust_amd ablate` (PACK_ABLATE=n builds; their outputs are
wrong by design — timing only).

    python3 scripts/ablate.py [--rounds R] [--iters K] [lib.so ...]
"""
import argparse
import ctypes as C
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def load(path):
    L = C.CDLL(path)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
    L.capnp_ctx_create.restype = vp
    L.capnp_gpu_pack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
    L.capnp_gpu_unpack_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    if hasattr(L, "capnp_gpu_unpack_batch_tuned"):
        L.capnp_gpu_unpack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, u32, vp]
    L.capnp_ctx_reserve.argtypes = [vp, sz]
    L.capnp_pack_tile_words.restype = C.c_uint32
    if hasattr(L, "capnp_unpack_tile_words"):
        L.capnp_unpack_tile_words.restype = C.c_uint32
    st = C.c_int(0)
    ctx = L.capnp_ctx_create(0, C.byref(st))
    assert ctx, st.value
    return L, C.c_void_p(ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--tc", type=int, default=0)
    ap.add_argument("--utc", type=int, default=0, help="unpack chunks per tile")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    libs = a.libs or ([os.path.join(ROOT, "capnproto-rust_amd/capnp_amd/libcapnp_packed.so")] +
                      sorted(glob.glob(os.path.join(ROOT, "capnproto-rust_amd/build/abl/*.so"))))
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    cap = ctx.batch_bound_bytes(n * cw, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ref_out, ref_oo = ctx.pack_batch(words, offs)
    packed = ref_out.clone()
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    variants = [(os.path.basename(p), *load(p)) for p in libs]
    for _, L, h in variants:
        L.capnp_ctx_reserve(h, n)
    res = {name: {"pack": [], "unpack": []} for name, _, _ in variants}
    P = C.c_void_p
    for r in range(a.rounds):
        for name, L, h in variants:
            for kind in ("pack", "unpack"):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.iters):
                    if kind == "pack":
                        tc = a.tc or tile_chunks_for(n * cw, n, L)
                        L.capnp_gpu_pack_batch_tuned(h, P(words.data_ptr()), P(offs.data_ptr()), n,
                                                     P(out.data_ptr()), cap, P(oo.data_ptr()), tc,
                                                     P(stream.cuda_stream))
                    else:
                        if hasattr(L, "capnp_gpu_unpack_batch_tuned"):
                            L.capnp_gpu_unpack_batch_tuned(
                                h, P(packed.data_ptr()), P(ref_oo.data_ptr()), n,
                                P(back.data_ptr()), P(offs.data_ptr()), P(status.data_ptr()),
                                None, a.utc or unpack_tile_chunks_for(n * cw, n, L),
                                P(stream.cuda_stream))
                        else:
                            L.capnp_gpu_unpack_batch(h, P(packed.data_ptr()), P(ref_oo.data_ptr()),
                                                     n, P(back.data_ptr()), P(offs.data_ptr()),
                                                     P(status.data_ptr()), None,
                                                     P(stream.cuda_stream))
                e1.record(stream)
                e1.synchronize()
                res[name][kind].append(e0.elapsed_time(e1) / a.iters)
    U = n * cw * 8
    for name, d in res.items():
        pm, um = statistics.median(d["pack"]), statistics.median(d["unpack"])
        print(f"{name:36s} pack {pm * 1e3:8.1f} us ({U / pm / 1e6:7.1f} GB/s U)   "
              f"unpack {um * 1e3:8.1f} us ({U / um / 1e6:7.1f} GB/s U)")


if __name__ == "__main__":
    main()
