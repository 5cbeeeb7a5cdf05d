#!/usr/bin/env python3
"""Per-tile phase timeline of the resync tile resolution's spec launch
(k_tile; build: make -C capnproto-rust_amd variant FILE=resync NAME=rprof
DEFS=-DRESYNC_PROF=1): staging + chunk search, spec walks, the rounds,
the look-back wait and re-run, block write-out (s_memrealtime, 100 MHz).  Diagnostic.

    python3 scripts/resync_prof.py [--lib path] [--workload config4_1GiB]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_rprof.so"))
    ap.add_argument("--workload", default="config4_1GiB")
    a = ap.parse_args()
    os.environ["CAPNP_PACKED_LIB"] = a.lib
    import torch
    from capnp_amd import Context, _lib
    import resync_bench as RB
    ctx = Context(0)
    words, offs, packed, poffs = RB.workload(ctx, a.workload)
    L = _lib.lib()
    L.capnp_resync_trace.argtypes = [C.c_void_p]
    nbytes = int(poffs[-1])
    ntiles = nbytes // (512 * 64) + len(poffs) // 64 + 64
    trace = torch.zeros(ntiles * 8, dtype=torch.int64, device="cuda")
    assert L.capnp_resync_trace(C.c_void_p(trace.data_ptr())) == 0
    out = torch.empty_like(words)
    st = torch.empty(len(poffs) - 1, dtype=torch.int32, device="cuda")
    for it in range(3):
        trace.zero_()
        ctx.unpack_batch_resync_into(packed, poffs, offs, out, st)
        torch.cuda.synchronize()
    assert torch.equal(out, words) and int(st.abs().sum()) == 0
    T = trace.view(ntiles, 8).cpu().numpy().astype(np.int64)
    T = T[T[:, 5] > 0]
    names = ["stage+search", "spec", "rounds", "wait+rerun", "write"]
    d = [(T[:, k + 1] - T[:, k]) / 100.0 for k in range(5)]
    span = (T[:, 5].max() - T[:, 0].min()) / 100.0
    life = (T[:, 5] - T[:, 0]) / 100.0
    print(f"tiles {len(T)}  span {span:.1f} us  lifetime mean {life.mean():.2f} p50 {np.median(life):.2f} p90 {np.percentile(life, 90):.2f} us")
    print("  mean us: " + "  ".join(f"{n} {x.mean():.2f}" for n, x in zip(names, d)))
    print("  p90 us : " + "  ".join(f"{n} {np.percentile(x, 90):.2f}" for n, x in zip(names, d)))
    print(f"  tiles in flight (sum of lifetimes / span): {life.sum() / span:.0f}")


if __name__ == "__main__":
    main()
