#!/usr/bin/env python3
"""Per-call latency of the drop-in message calls (capnp_packed_write_message /
capnp_packed_read_message, one message per call as the reference's
`benchmark carsales bytes reuse packed` makes them, benchmark.rs:207-259):
median and 10th percentile over many calls, write and read separately, for
one-segment messages of config-2 words of several sizes.

    python3 scripts/percall_bench.py [--reps N] [--lib PATH]

--lib loads a library variant; one built with -DSVC_PROF=1 also reports
the resident services' per-request phases (bell seen -> arguments in, and
the body), averaged per size.  CAPNP_PERCALL_SERVICE=0 launches every call.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--sizes", default="128,512,1500,2048,8192,32768",
                    help="message words, comma-separated")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401
    import oracle_lib as O
    from capnp_amd import Context, _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    L = _lib.lib()
    prof = []
    for name, kind in (("capnp_svc_prof", "read"), ("capnp_svc_prof_w", "write")):
        try:
            f = getattr(L, name)
            f.restype = C.c_int
            prof.append((f, kind))
        except AttributeError:
            pass
    p8 = (C.c_ulonglong * 24)()
    ctx = Context(0)
    h = ctx.handle
    opts = _lib.ReaderOptionsC(0, 0, 64)
    rows = []
    for words in [int(x) for x in a.sizes.split(",")]:
        offs = np.array([0, words], np.uint64)
        seg = O.gen_fill(offs, kind0=0, pz=O.PZ30)
        ptrs = (C.c_void_p * 1)(seg.ctypes.data)
        lens = (C.c_uint32 * 1)(words)
        cap = L.capnp_packed_batch_bound_bytes(words + 1, 3)
        out = np.empty(cap, np.uint8)
        body = np.empty(words, np.uint64)
        segs = np.empty(512, np.uint32)
        n, used, nseg = C.c_size_t(0), C.c_size_t(0), C.c_uint32(0)
        tw, tr = [], []
        for f, _ in prof:
            f(p8, 1)
        for r in range(a.reps + 10):
            t0 = time.perf_counter()
            st = L.capnp_packed_write_message(h, ptrs, lens, 1, out.ctypes.data, cap, C.byref(n))
            t1 = time.perf_counter()
            st2 = L.capnp_packed_read_message(h, out.ctypes.data, n.value, C.byref(opts), 0,
                                              body.ctypes.data, words, segs.ctypes.data,
                                              C.byref(nseg), C.byref(used))
            t2 = time.perf_counter()
            assert st == 0 and st2 == 0 and used.value == n.value
            if r >= 10:
                tw.append(t1 - t0)
                tr.append(t2 - t1)
        assert np.array_equal(body, seg)
        st, ref = O.write_message([seg])
        assert bytes(out[:n.value]) == ref
        tw, tr = np.array(tw) * 1e6, np.array(tr) * 1e6
        r = {"words": words, "kib": words * 8 / 1024, "packed_bytes": n.value,
             "write_us_median": round(float(np.median(tw)), 1),
             "write_us_p10": round(float(np.percentile(tw, 10)), 1),
             "read_us_median": round(float(np.median(tr)), 1),
             "read_us_p10": round(float(np.percentile(tr, 10)), 1)}
        for f, kind in prof:
            f(p8, 1)
            if p8[0]:
                r[kind + "_svc"] = {"requests": p8[0], "args_us": round(p8[1] / p8[0] / 100, 2),
                                    "body_us": round(p8[2] / p8[0] / 100, 2),
                                    "body_clock_mhz": round(100 * p8[8] / max(p8[2], 1))}
                if kind == "write" and p8[6]:
                    r["write_phases_us"] = {
                        "stage": round((p8[6] - p8[7]) / p8[0] / 100, 2),
                        "sizes": round(p8[3] / p8[0] / 100, 2),
                        "scan": round(p8[4] / p8[0] / 100, 2),
                        "pass_b": round(p8[5] / p8[0] / 100, 2),
                        "copy_out": round(p8[9] / p8[0] / 100, 2)}
                if kind == "read" and p8[6]:
                    r["read_phases_us"] = {
                        "stage": round((p8[6] - p8[7]) / p8[0] / 100, 2),
                        "table": round(p8[3] / p8[0] / 100, 2),
                        "decode": round(p8[4] / p8[0] / 100, 2),
                        "results_landed": round(p8[5] / p8[0] / 100, 2)}
                    if p8[12]:
                        r["read_small_us"] = {"n": p8[12],
                                              "sel_init": round(p8[9] / p8[12] / 100, 2),
                                              "walk": round(p8[10] / p8[12] / 100, 2),
                                              "expand": round(p8[11] / p8[12] / 100, 2),
                                              "spec": round(p8[16] / p8[12] / 100, 2),
                                              "rounds": round(p8[17] / p8[12] / 100, 2),
                                              "last_walk": round(p8[18] / p8[12] / 100, 2),
                                              "descriptors": round(p8[19] / p8[12] / 100, 2),
                                              "rounds_taken": round(p8[20] / p8[12], 2)}
                    if p8[23] >> 32:
                        k = p8[23] >> 32
                        r["read_mid_us"] = {"n": k,
                                            "spec": round(p8[13] / k / 100, 2),
                                            "passes": round(p8[14] / k / 100, 2),
                                            "words": round(p8[15] / k / 100, 2),
                                            "descriptors": round(p8[21] / k / 100, 2),
                                            "expand": round(p8[22] / k / 100, 2),
                                            "passes_taken": round((p8[23] & 0xFFFFFFFF) / k, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
