#!/usr/bin/env python3
"""Diagnostic: one read_message case of tests/test_gpu_long_units.py's
mid-size cases (by input length, argv[1]; default the misaligned-table case)
through the library named by CAPNP_PACKED_LIB, against the oracle."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
import oracle_lib as O  # noqa: E402


def _packed(words):
    return O.pack(np.asarray(words, np.uint64).tobytes())[1]


def mid_cases():
    rng = np.random.default_rng(33)
    cases = []
    for k in (560, 600, 700, 900, 1024, 1500, 1800, 2000, 2200, 2400, 8192):
        for kind in (0, 1, 2):
            w = O.gen_fill(np.array([0, k], np.uint64), kinds=np.array([kind], np.uint8),
                           pz=O.PZ30, id0=1900 + k + kind)
            msg = O.write_message([w])[1]
            cases += [msg, msg + O.write_message([w[:3]])[1], msg[:len(msg) - 1],
                      msg[:max(9, len(msg) // 2)], _packed([(k - 1) << 32]) + _packed(w)]
            bad = bytearray(msg)
            bad[8 + int(rng.integers(0, len(msg) - 8))] ^= 0x5A
            cases.append(bytes(bad))
    for k in (800, 1500, 2000):
        w = np.zeros(k, np.uint64)
        a, b = k // 4 - 7, k // 2 + 5
        w[:a] = 0x0102030405060708
        w[b:] = 0x1112131415161718
        w[rng.integers(0, k, 5)] = 0x0000000400000001
        cases.append(O.write_message([w])[1])
    for i in range(30):
        k = int(rng.integers(500, 2000))
        body = rng.integers(0, 256, int(rng.integers(5200, 16000))).astype(np.uint8).tobytes()
        cases.append(_packed([k << 32]) + body)
    return cases


def main():
    import torch
    from capnp_amd import Context, _lib
    L = _lib.lib()
    ctx = Context(0)
    opts = _lib.ReaderOptionsC(0, 0, 64)
    want = int(sys.argv[1]) if len(sys.argv) > 1 else 5681
    for data in mid_cases():
        if len(data) != want:
            continue
        d = np.frombuffer(data, np.uint8).copy()
        cap = len(d) * 128 + 64
        body = np.zeros(cap + 1, np.uint64)
        sw = np.zeros(512, np.uint32)
        ns, used = C.c_uint32(0), C.c_size_t(0)
        r = L.capnp_packed_read_message(ctx.handle, d.ctypes.data, len(d), C.byref(opts), 0,
                                        body.ctypes.data, cap + 1, sw.ctypes.data, C.byref(ns),
                                        C.byref(used))
        torch.cuda.synchronize()
        rst, rsegs, rused = O.read_message(data)
        print("len", len(data), "gpu", r, used.value, "oracle", rst, rused, flush=True)


if __name__ == "__main__":
    main()
