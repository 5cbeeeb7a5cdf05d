#!/usr/bin/env python3
"""Diagnostic: the index-free batch unpack (fit + overflow kernels) on
batches of one chunk kind and size, packed by the library; prints the
round-trip check and the unpack time per call (HIP events).  Used to find
what the overflow kernel spends its time on in config 4's block decode.

    python3 scripts/ovf_probe.py [lib.so]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, ROOT)


def main():
    if len(sys.argv) > 1:
        os.environ["CAPNP_PACKED_LIB"] = sys.argv[1]
        print("lib", sys.argv[1])
    import torch
    import bench
    from capnp_amd import Context
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    for kind, cw, n in ((1, 8192, 2300), (1, 2048, 2300), (1, 8192, 256), (0, 128, 70000),
                        (2, 128, 70000)):
        offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
        words = torch.empty(n * cw, dtype=torch.int64, device=dev)
        kinds = torch.full((n,), kind, dtype=torch.uint8, device=dev)
        ctx.gen_batch(words, offs, pz_thresh=bench.PZ["config4"], kinds=kinds)
        packed, poffs = ctx.pack_batch(words, offs)
        back = torch.empty_like(words)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        for tc in (16, 1):
            for _ in range(3):
                ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tc)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tc)
            e1.record()
            e1.synchronize()
            ok = torch.equal(back, words) and int(st.abs().sum()) == 0
            print(f"kind {kind} chunk {cw} words x {n}: packed {int(poffs[-1])} B, tc {tc}: "
                  f"{e0.elapsed_time(e1) / 5 * 1e3:.1f} us ok {ok}", flush=True)


if __name__ == "__main__":
    main()
