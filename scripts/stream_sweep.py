#!/usr/bin/env python3
"""Host-to-host rates of the streaming batch API (capnp_stream_*) for several
slice sizes on the config-2 batch, next to the sequential copy-kernel-copy
path (diagnostic).

    python3 scripts/stream_sweep.py [--slices 4,8,16,32,64]   (Mi words)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--slices", default="4,8,16,32,64")
    a = ap.parse_args()
    import torch
    from capnp_amd import Context
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=1288490189)
    U = n * cw * 8
    h_words = words.cpu().pin_memory()
    h_offs = offs.cpu().pin_memory()
    cap = ctx.batch_bound_bytes(n * cw, n)
    h_packed = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    h_poffs = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
    h_back = torch.empty_like(h_words).pin_memory()
    h_status = torch.empty(n, dtype=torch.int32, pin_memory=True)
    for sw in [int(x) << 20 for x in a.slices.split(",")]:
        enc, dec = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.stream_pack(h_words, h_offs, h_packed, h_poffs, slice_words=sw)
            t1 = time.perf_counter()
            ctx.stream_unpack(h_packed, h_poffs, h_offs, h_back, h_status, slice_words=sw)
            t2 = time.perf_counter()
            enc.append(t1 - t0)
            dec.append(t2 - t1)
        ok = torch.equal(h_back, h_words) and int(h_status.sum()) == 0
        print(f"slice {sw >> 20:3d} Mi words: encode {U / min(enc) / GiB:6.2f} GiB/s, "
              f"decode {U / min(dec) / GiB:6.2f} GiB/s ok={ok}", flush=True)
    # raw copy rates for reference
    d = torch.empty_like(words)
    for name, fn in (("H2D 1 GiB", lambda: d.copy_(h_words, non_blocking=True)),
                     ("D2H 1 GiB", lambda: h_back.copy_(d, non_blocking=True))):
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"{name}: {U / min(ts) / GiB:6.2f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
