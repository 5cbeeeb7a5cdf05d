#!/usr/bin/env python3
"""Index-free decode of long read units, one chunk per workgroup
(chunks_per_tile=1: every chunk too large for the tile tables takes the
overflow kernels' long-unit path, csrc/unpack.hip unpack_long), by generator
kind and chunk size: round-trip check and the unpack time per call (HIP
events on the stream the kernels run on).  Round 4's single-wave walk took
27.2 ms for 256 x 8192-word kind-0 chunks (profiles/r04g3_global1_walk32.txt).

    python3 scripts/long_unit_bench.py [lib.so] [--auto]

--auto: chunks_per_tile=0, the library's own choice (a batch whose mean
chunk is >= 512 words takes the index-free block decode, resync.hip, which
spreads one long unit over the whole chip); plus one 8 Mi-word unit.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, ROOT)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    auto = "--auto" in sys.argv[1:]
    if args:
        os.environ["CAPNP_PACKED_LIB"] = args[0]
    import torch
    import bench
    from capnp_amd import Context
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    rows = []
    cases = ((0, 8192, 256), (1, 8192, 256), (2, 8192, 256), (0, 2560, 256),
             (0, 65536, 64), (0, 1 << 20, 2), (1, 1 << 20, 2), (0, 8192, 2300))
    if auto:
        cases = cases + ((0, 1 << 23, 1), (2, 1 << 23, 1), (0, 1 << 20, 1))
    tpc = 0 if auto else 1
    for kind, cw, n in cases:
        offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
        words = torch.empty(n * cw, dtype=torch.int64, device=dev)
        kinds = torch.full((n,), kind, dtype=torch.uint8, device=dev)
        ctx.gen_batch(words, offs, pz_thresh=bench.PZ["config4"], kinds=kinds)
        packed, poffs = ctx.pack_batch(words, offs)
        back = torch.empty_like(words)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream()
        for _ in range(2):
            ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tpc)
        torch.cuda.synchronize()
        back.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            ctx.unpack_batch_into(packed, poffs, offs, back, st, chunks_per_tile=tpc)
        e1.record(s)
        e1.synchronize()
        ok = torch.equal(back, words) and int(st.abs().sum()) == 0
        us = e0.elapsed_time(e1) / reps * 1e3
        r = {"mode": "auto" if auto else "tc1", "kind": kind, "chunk_words": cw, "chunks": n,
             "packed_bytes": int(poffs[-1]),
             "us": round(us, 1), "GiBps_unpacked": round(n * cw * 8 / us / 1e3 / 1.073741824, 2),
             "ok": bool(ok)}
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
