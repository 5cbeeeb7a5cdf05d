#!/usr/bin/env python3
"""Throughput of capnp_gpu_write_messages / capnp_gpu_read_messages on config-2-shaped batches (1 Mi
single-segment 1 KiB messages), next to the plain chunk batch pack of the
same words (diagnostic).

    python3 scripts/msg_bench.py [--msgs N] [--segs-per-msg S]
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
    ap.add_argument("--msgs", type=int, default=1 << 20)
    ap.add_argument("--segs-per-msg", type=int, default=1)
    ap.add_argument("--words", type=int, default=128)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context
    ctx = Context(0)
    nm, sp, cw = a.msgs, a.segs_per_msg, a.words
    nseg = nm * sp
    seg_off = torch.arange(0, (nseg + 1) * (cw // sp), cw // sp, dtype=torch.int64, device="cuda")
    words = torch.empty(int(seg_off[-1]), dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, seg_off, pz_thresh=1288490189)
    msg_off = torch.arange(0, (nm + 1) * sp, sp, dtype=torch.int64, device="cuda")
    U = words.numel() * 8
    packed, mo = ctx.write_messages(words, seg_off, msg_off)
    pk, po = ctx.pack_batch(words, seg_off)
    torch.cuda.synchronize()
    for name, fn in (("write_messages", lambda: ctx.write_messages(words, seg_off, msg_off)),
                     ("pack_batch (chunks only)", lambda: ctx.pack_batch(words, seg_off)),
                     ("read_messages", lambda: ctx.read_messages(packed, mo, words.numel(), nseg)),
                     ("unpack_batch (chunks only)", lambda: ctx.unpack_batch(pk, po, seg_off))):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        if name == "read_messages":
            r = fn()
            torch.cuda.synchronize()
            assert int((r[4] != 0).sum()) == 0 and torch.equal(r[0][:words.numel()], words)
        print(f"{name}: {min(ts) * 1e3:.3f} ms, {U / min(ts) / GiB:.1f} GiB/s of segment words",
              flush=True)


if __name__ == "__main__":
    main()
