#!/usr/bin/env python3
"""Probe: the index-free batch decode of a workload (default config4) through
the chunk-tile path at several chunks-per-tile (tiles that fit the LDS tables
are staged, longer chunks take the long-unit decode, one workgroup each)
against the library's own choice (chunks_per_tile=0: the resync block decode
for a mean chunk of >= 512 words).  Round trip checked; us per call.
Diagnostic only.

    python3 scripts/route_probe.py [--wl=config4]
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
    wl = "config4"
    for a in sys.argv[1:]:
        if a.startswith("--wl="):
            wl = a[5:]
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    args = bench.parse(["--workload", wl])
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    packed, poffs = ctx.pack_batch(words, offs)
    back = torch.empty_like(words)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    print(f"{wl}: {n} chunks, {words.numel()} words, {int(poffs[-1])} packed bytes", flush=True)
    tcs = [int(x) for x in os.environ.get("TCS", "0,1,2,4,8,16").split(",")]
    for tc in tcs:
        for _ in range(3):
            ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tc)
        torch.cuda.synchronize()
        back.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tc)
        e1.record(s)
        e1.synchronize()
        ok = torch.equal(back, words) and int(st.abs().sum()) == 0
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"chunks_per_tile={tc}: {us:8.1f} us  {words.numel() * 8 / us / 1e3 / 1.073741824:7.1f}"
              f" GiB/s  ok={ok}", flush=True)


if __name__ == "__main__":
    main()
