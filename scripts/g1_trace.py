#!/usr/bin/env python3
"""Diagnostic: per-chunk cycles of the overflow path's global walk
(unpack_global1) from the UNPACK_PROF=1 build (make -C capnproto-rust_amd
variant FILE=unpack NAME=uprof DEFS=-DUNPACK_PROF=1): total, walk (wave 0,
with the barriers around it) and expansion s_memtime cycles and windows per
chunk, for 256 chunks of 8192 words of each generator kind, decoded one
chunk per tile.

    python3 scripts/g1_trace.py
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, ROOT)
os.environ["CAPNP_PACKED_LIB"] = os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_uprof.so")


def main():
    import torch
    import bench
    from capnp_amd import Context, _lib
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    L.capnp_unpack_trace.argtypes = [C.c_void_p]
    for kind, cw, n in ((1, 8192, 256), (2, 8192, 256), (0, 8192, 256)):
        offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
        words = torch.empty(n * cw, dtype=torch.int64, device=dev)
        kinds = torch.full((n,), kind, dtype=torch.uint8, device=dev)
        ctx.gen_batch(words, offs, pz_thresh=bench.PZ["config4"], kinds=kinds)
        packed, poffs = ctx.pack_batch(words, offs)
        back = torch.empty_like(words)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        tr = torch.zeros(4 * n, dtype=torch.int64, device=dev)
        assert L.capnp_unpack_trace(C.c_void_p(tr.data_ptr())) == 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = torch.equal(back, words) and int(st.abs().sum()) == 0
        t = tr.view(n, 4).float().mean(0).tolist()
        print(f"kind {kind} {cw} words x {n}: packed {int(poffs[-1]) // n} B/chunk ok {ok} "
              f"call {dt * 1e6:.0f} us: cycles total {t[0]:.0f} walk {t[1]:.0f} "
              f"expand {t[2]:.0f} windows {t[3]:.1f}", flush=True)
        L.capnp_unpack_trace(None)


if __name__ == "__main__":
    main()
