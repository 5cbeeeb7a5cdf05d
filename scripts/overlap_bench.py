#!/usr/bin/env python3
"""Does pack of batch i + 1 overlap unpack of batch i?  Config-2 round trips
(bench.py's kernels and tile sizes, record sync index) timed two ways after
the clocks settle:

  sequential  pack, unpack, pack, ... on one stream (bench.py's step)
  overlapped  packs on stream A, unpacks on stream B, two packed buffers:
              unpack i waits for pack i, pack i + 2 for unpack i

Prints ms per round trip and GiB/s for each, best of 3 blocks of K steps.
Diagnostic."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    import bench
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    args = bench.parse(["--workload", os.environ.get("WL", "config2")])
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    total = words.numel()
    cap = ctx.batch_bound_bytes(total, n)
    packed = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
    poffs = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    sync = [torch.empty(ctx.sync_entries(total), dtype=torch.int32, device=dev) for _ in range(2)]
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    tc = tile_chunks_for(total, n)
    utc = unpack_tile_chunks_for(total, n, sync=True)
    ctx.reserve(n)
    sA = torch.cuda.Stream(device=dev)
    sB = torch.cuda.Stream(device=dev)
    U = total * 8

    def seq(k):
        s = torch.cuda.current_stream()
        for _ in range(k):
            ctx.pack_batch_into(words, offs, packed[0], poffs[0], chunks_per_tile=tc, sync=sync[0],
                                stream=s.cuda_stream)
            ctx.unpack_batch_into(packed[0], poffs[0], offs, back, status, chunks_per_tile=utc,
                                  sync=sync[0], stream=s.cuda_stream)

    def ovl(k):
        packed_ev = [torch.cuda.Event() for _ in range(k)]
        used_ev = [torch.cuda.Event() for _ in range(k)]
        for i in range(k):
            b = i % 2
            if i >= 2:
                sA.wait_event(used_ev[i - 2])
            ctx.pack_batch_into(words, offs, packed[b], poffs[b], chunks_per_tile=tc, sync=sync[b],
                                stream=sA.cuda_stream)
            packed_ev[i].record(sA)
            sB.wait_event(packed_ev[i])
            ctx.unpack_batch_into(packed[b], poffs[b], offs, back, status, chunks_per_tile=utc,
                                  sync=sync[b], stream=sB.cuda_stream)
            used_ev[i].record(sB)

    def timed(f, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f(k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    t_end = time.perf_counter() + 0.08  # settle the clocks
    while time.perf_counter() < t_end:
        seq(8)
        torch.cuda.synchronize()
    for name, f in (("sequential", seq), ("overlapped", ovl), ("sequential", seq),
                    ("overlapped", ovl)):
        best = min(timed(f, K) for _ in range(3))
        ok = torch.equal(back, words) and int((status != 0).sum()) == 0
        print(f"{name:11s} {best / K * 1e3:.4f} ms per round trip  {U / (best / K) / 2**30:8.1f} GiB/s  "
              f"ok={ok}", flush=True)


if __name__ == "__main__":
    main()
