#!/usr/bin/env python3
"""Per-step kernel times of the headline round trip over a long run (the
GPU's clock/power transient after idle): pack and unpack durations of each
step with HIP events, plus the GPU's reported clocks every few steps.
Diagnostic only.

    python3 scripts/clock_curve.py [--steps N] [--idle-ms T] [--workload W]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def clocks():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True,
                           timeout=10)
        d = json.loads(r.stdout)
        c = next(iter(d.values()))
        return {k: v for k, v in c.items() if "clock" in k.lower()}
    except Exception as e:  # (diagnostic: any failure is just reported)
        return {"err": str(e)[:80]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--idle-ms", type=int, default=300)
    ap.add_argument("--workload", default="config2")
    a = ap.parse_args()
    import bench
    import torch
    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    args = bench.parse(["--workload", a.workload])
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    words, offs, n, _ = bench.make_workload(args, ctx, torch, dev, 0)
    total = words.numel()
    packed = torch.empty(ctx.batch_bound_bytes(total, n), dtype=torch.uint8, device=dev)
    poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    sync = torch.empty(ctx.sync_entries(total), dtype=torch.int32, device=dev)
    tc = tile_chunks_for(total, n)
    utc = unpack_tile_chunks_for(total, n, sync=True)
    ctx.reserve(n)
    s = torch.cuda.current_stream()
    for rnd in range(2):
        torch.cuda.synchronize()
        time.sleep(a.idle_ms / 1e3)
        print(f"round {rnd} after {a.idle_ms} ms idle; clocks {clocks()}", flush=True)
        ev = []
        t0 = time.perf_counter()
        for i in range(a.steps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(s)
            ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tc, sync=sync)
            e[1].record(s)
            ctx.unpack_batch_into(packed, poffs, offs, back, status, chunks_per_tile=utc, sync=sync)
            e[2].record(s)
            ev.append(e)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"  clocks after: {clocks()}", flush=True)
        p = [e[0].elapsed_time(e[1]) * 1e3 for e in ev]
        u = [e[1].elapsed_time(e[2]) * 1e3 for e in ev]
        print(f"  wall {wall * 1e3:.1f} ms for {a.steps} steps; ok {torch.equal(back, words)}")
        for k in range(0, a.steps, 10):
            print(f"  steps {k:3d}-{k + 9:3d}: pack " + " ".join(f"{x:4.0f}" for x in p[k:k + 10])
                  + " | unpack " + " ".join(f"{x:4.0f}" for x in u[k:k + 10]), flush=True)


if __name__ == "__main__":
    main()
