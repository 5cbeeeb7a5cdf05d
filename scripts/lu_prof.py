#!/usr/bin/env python3
"""Diagnostic: phases of the long-unit decode (csrc/unpack.hip unpack_long)
from the UNPACK_PROF build (make -C capnproto-rust_amd variant FILE=unpack
NAME=uprof DEFS=-DUNPACK_PROF=1): per window, microseconds in stage, spec
walk, rounds (and their count), words (+ the last segment's walk) and
descriptors + expansion, for read_message calls of one-segment messages
(msg_read_kernel) and for batches of long chunks (the overflow kernel).

    python3 scripts/lu_prof.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
os.environ["CAPNP_PACKED_LIB"] = os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_uprof" + os.environ.get("LUPROF", "") + ".so")


def show(tag, L):
    v = (C.c_ulonglong * 16)()
    assert L.capnp_unpack_prof(v, 1) == 0
    nw = max(v[1], 1)
    if v[8] or v[0]:
        print(f"{tag}: overflow tiles {v[8]} ({v[9] / max(v[8], 1) / 100:.2f} us each), "
              f"serial chunk walks {v[0]}", flush=True)
    print(f"{tag}: windows {v[1]} rounds/window {v[2] / nw:.2f} us/window: stage {v[3] / nw / 100:.2f} "
          f"spec {v[4] / nw / 100:.2f} rounds {v[5] / nw / 100:.2f} words {v[6] / nw / 100:.2f} "
          f"desc+expand {v[7] / nw / 100:.2f}", flush=True)


def reset(L):
    v = (C.c_ulonglong * 16)()
    assert L.capnp_unpack_prof(v, 1) == 0


def main():
    import torch
    import oracle_lib as O
    import bench
    from capnp_amd import Context, _lib
    L = _lib.lib()
    L.capnp_unpack_prof.argtypes = [C.c_void_p, C.c_int]
    ctx = Context(0)
    h = ctx.handle
    opts = _lib.ReaderOptionsC(0, 0, 64)
    for words in (128, 1500, 8192):
        offs = np.array([0, words], np.uint64)
        seg = O.gen_fill(offs, kind0=0, pz=O.PZ30)
        st, msg = O.write_message([seg])
        buf = np.frombuffer(msg, np.uint8).copy()
        body = np.empty(words, np.uint64)
        segs = np.empty(512, np.uint32)
        used, nseg = C.c_size_t(0), C.c_uint32(0)
        reset(L)
        for _ in range(5):
            L.capnp_packed_read_message(h, buf.ctypes.data, len(buf), C.byref(opts), 0,
                                        body.ctypes.data, words, segs.ctypes.data, C.byref(nseg),
                                        C.byref(used))
        assert np.array_equal(body, seg)
        show(f"read_message {words} words", L)
    dev = torch.device("cuda", 0)
    for kind, cw, n in ((0, 8192, 256), (1, 8192, 256), (2, 8192, 256)):
        offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
        w = torch.empty(n * cw, dtype=torch.int64, device=dev)
        kinds = torch.full((n,), kind, dtype=torch.uint8, device=dev)
        ctx.gen_batch(w, offs, pz_thresh=bench.PZ["config4"], kinds=kinds)
        packed, poffs = ctx.pack_batch(w, offs)
        back = torch.empty_like(w)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        reset(L)
        ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=1)
        torch.cuda.synchronize()
        assert torch.equal(back, w)
        show(f"batch kind {kind} {cw} words x {n}", L)
    # config 4 without the index: the resync block decode hands the blocks
    # that expand past a tile (zero-run blocks) to the long-unit decode
    args = bench.parse(["--workload", "config4"])
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    packed, poffs = ctx.pack_batch(words, offs)
    torch.cuda.synchronize()
    reset(L)
    back, st, _ = ctx.unpack_batch(packed, poffs, offs)
    torch.cuda.synchronize()
    assert torch.equal(back, words)
    show("config 4 index-free (overflow blocks)", L)


if __name__ == "__main__":
    main()
