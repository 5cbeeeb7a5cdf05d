#!/usr/bin/env python3
"""Runs pack and unpack of the config-2 workload a few times (for rocprofv3
counter passes that should see only the codec kernels)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--chunk-words", type=int, default=128)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    n, cw = a.chunks, a.chunk_words
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    cap = ctx.batch_bound_bytes(n * cw, n)
    packed = torch.empty(cap, dtype=torch.uint8, device="cuda")
    poffs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    tc, utc = tile_chunks_for(n * cw, n), unpack_tile_chunks_for(n * cw, n)
    ctx.reserve(n)
    for _ in range(a.iters):
        ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tc)
        ctx.unpack_batch_into(packed, poffs, offs, back, status, chunks_per_tile=utc)
    torch.cuda.synchronize()
    assert torch.equal(back, words)
    print("ok")


if __name__ == "__main__":
    main()
