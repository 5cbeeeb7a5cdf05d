#!/usr/bin/env python3
"""Why a kernel times differently alone and inside the round trip: config-2
pack and unpack (with the record sync index, bench.py's kernels and tile
sizes), each timed with HIP events

  alone      the same kernel 5 times back to back,
  roundtrip  pack, unpack, pack, ... (bench.py's step),
  after_w    each launch after a 1 GiB write of another buffer (the caches
             full of dirty lines, as after the other kernel of the round trip)
  after_r    each launch after a 1 GiB read of another buffer (clean caches).

Prints µs per launch.  Diagnostic."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    import bench
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    args = bench.parse(["--workload", os.environ.get("WL", "config2")])
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    total = words.numel()
    packed = torch.empty(ctx.batch_bound_bytes(total, n), dtype=torch.uint8, device=dev)
    poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    sync = torch.empty(ctx.sync_entries(total), dtype=torch.int32, device=dev)
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    scratch = torch.empty(1 << 27, dtype=torch.int64, device=dev)  # 1 GiB
    tc = tile_chunks_for(total, n)
    utc = unpack_tile_chunks_for(total, n, sync=True)
    stream = torch.cuda.current_stream()

    def pack():
        ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tc, sync=sync)

    def unpack():
        ctx.unpack_batch_into(packed, poffs, offs, back, status, chunks_per_tile=utc, sync=sync)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        return e0, e1

    res = {}
    for rep in range(3):
        for name, seq in (
                ("alone", [("pack", None)] * 5 + [("unpack", None)] * 5),
                ("roundtrip", [("pack", None), ("unpack", None)] * 5),
                ("after_w", [("pack", "w"), ("unpack", "w")] * 5),
                ("after_r", [("pack", "r"), ("unpack", "r")] * 5)):
            ev = []
            for k, pre in seq:
                if pre == "w":
                    scratch.fill_(7)
                elif pre == "r":
                    scratch.sum()
                ev.append((k, timed(pack if k == "pack" else unpack)))
            torch.cuda.synchronize()
            for k, (e0, e1) in ev:
                res.setdefault((name, k), []).append(e0.elapsed_time(e1) * 1e3)
    assert torch.equal(back, words)
    for (name, k), v in sorted(res.items()):
        print(f"{name:10s} {k:7s} median {statistics.median(v):8.1f} us  min {min(v):8.1f}",
              flush=True)


if __name__ == "__main__":
    main()
