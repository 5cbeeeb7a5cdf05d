#!/usr/bin/env python3
"""Probe: one config-2 step (pack + unpack of 1 Mi x 1 KiB segments) cut into
N pieces, the unpack of piece i on a second stream overlapping the pack of
piece i + 1 (stream order plus one event per piece).  Prints ms per step
for N = 1, 2, 4, 8 and checks the round trip.  Diagnostic only.

    python3 scripts/pipe_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from capnp_amd import Context
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    args = bench.parse(["--workload", "config2"])
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    total = words.numel()
    for N in (1, 2, 4, 8):
        m = n // N
        pieces = []
        for k in range(N):
            c0, c1 = k * m, (k + 1) * m if k < N - 1 else n
            w = words[int(offs[c0]):int(offs[c1])]
            o = (offs[c0:c1 + 1] - offs[c0]).contiguous()
            cap = ctx.batch_bound_bytes(w.numel(), c1 - c0)
            pieces.append(dict(w=w, o=o, n=c1 - c0,
                               out=torch.empty(cap, dtype=torch.uint8, device=dev),
                               oo=torch.empty(c1 - c0 + 1, dtype=torch.int64, device=dev),
                               sync=torch.empty(ctx.sync_entries(w.numel()), dtype=torch.int32,
                                                device=dev),
                               back=torch.empty_like(w),
                               st=torch.empty(c1 - c0, dtype=torch.int32, device=dev),
                               ev=torch.cuda.Event()))
        sp = torch.cuda.Stream()
        su = torch.cuda.Stream()

        def step():
            for p in pieces:
                with torch.cuda.stream(sp):
                    ctx.pack_batch_into(p["w"], p["o"], p["out"], p["oo"], chunks_per_tile=16,
                                        sync=p["sync"], stream=sp.cuda_stream)
                    p["ev"].record(sp)
                su.wait_event(p["ev"])
                with torch.cuda.stream(su):
                    ctx.unpack_batch_into(p["out"], p["oo"], p["o"], p["back"], p["st"],
                                          chunks_per_tile=16, sync=p["sync"], stream=su.cuda_stream)
            sp.wait_stream(su)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        ok = all(torch.equal(p["back"], p["w"]) and int(p["st"].abs().sum()) == 0 for p in pieces)
        K = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(sp)
        for _ in range(K):
            step()
        e1.record(sp)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / K
        print(f"N={N}: {ms:.4f} ms/step  {total * 8 / 2**30 / ms * 1e3:.1f} GiB/s  ok={ok}",
              flush=True)


if __name__ == "__main__":
    main()
