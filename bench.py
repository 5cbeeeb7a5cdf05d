#!/usr/bin/env python3
"""Benchmark: packed encode+decode of device-resident Cap'n Proto segments.

Workload (BASELINE.json configs[1]): 1 Mi segments x 1 KiB (128 words) per
GPU, ~30 % zero words (SURVEY.md §8d config 2 generator), resident in HBM.
One step = PACK the whole batch (capnp_gpu_pack_batch) and UNPACK it back
(capnp_gpu_unpack_batch) — the encode+decode round trip of the metric.
value = unpacked GiB per step (all ranks) / step time.

Multi-GPU: one process per GPU (torch.distributed.run); every rank packs
and unpacks its own shard of independent segments (chunk ids offset by
rank), no data-path collective; scaling is weak.  RCCL is used only for the
barrier and the max-over-ranks of the timing.

The JSON line also carries
  roofline      the dominant kernel's algorithmic bytes per launch / its mean
                launch time (HIP events on the launch stream) vs 8 TB/s;
  cpu_baseline  the CPU oracle (C restatement of the reference codec) timed
                on a bounded sample of the same workload on this host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MEASURED_COPY_GBS = 6290.0  # measured float4 copy (same source)
PZ = {"config2": 1288490189, "config3": 3435973837}
METRIC = "GiB/s packed encode+decode, device-resident segments; % HBM roofline"
GiB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=1 << 20, help="segments per GPU")
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--workload", default="config2", choices=["config2", "config3"])
    ap.add_argument("--cpu-sample-chunks", type=int, default=1 << 18)
    ap.add_argument("--cpu-reps", type=int, default=4)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time host->device->host")
    ap.add_argument("--no-sync", action="store_true",
                    help="pack without the record sync index; unpack walks whole chunks")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle pack + unpack of the first `cpu_sample_chunks` segments of the
    same workload on this host's cores."""
    import numpy as np
    import oracle_lib as O
    n, cw = args.cpu_sample_chunks, args.chunk_words
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or \
        min(16, os.cpu_count() or 1)
    offs = np.arange(0, (n + 1) * cw, cw, dtype=np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=PZ[args.workload])

    def timed(nn, thr, reps):
        w, o = words[:nn * cw], offs[:nn + 1]
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            st, packed, poffs = O.pack_batch(w, o, threads=thr)
            t1 = time.perf_counter()
            back, status, _ = O.unpack_batch(packed, poffs, o, threads=thr)
            t2 = time.perf_counter()
            assert st == 0 and (status == 0).all() and np.array_equal(back, w)
            if best is None or t2 - t0 < best[0]:
                best = (t2 - t0, t1 - t0, t2 - t1)
        return best

    best = timed(n, threads, args.cpu_reps)
    n1 = max(1, n // 16)
    one = timed(n1, 1, 2)
    u = n * cw * 8
    u1 = n1 * cw * 8
    return {
        "value": round(u / best[0] / GiB, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} segments x {cw * 8} B ({u / GiB:.3f} GiB) of the same generator, "
                  f"pack+unpack, best of {args.cpu_reps}, {threads} threads "
                  f"(oracle/packed_oracle.c, gcc -O3)",
        "pack_gibps": round(u / best[1] / GiB, 3),
        "unpack_gibps": round(u / best[2] / GiB, 3),
        "single_thread_gibps": round(u1 / one[0] / GiB, 3),
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    ctx = Context(local)
    n, cw = args.chunks, args.chunk_words
    total_words = n * cw
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
    words = torch.empty(total_words, dtype=torch.int64, device=dev)
    ctx.gen_batch(words, offs, pz_thresh=PZ[args.workload], id0=rank * n)
    cap = ctx.batch_bound_bytes(total_words, n)
    packed = torch.empty(cap, dtype=torch.uint8, device=dev)
    poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    back = torch.empty(total_words, dtype=torch.int64, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    consumed = torch.empty(n, dtype=torch.int64, device=dev)
    sync = None
    if not args.no_sync:
        sync = torch.empty(ctx.sync_entries(total_words), dtype=torch.int32, device=dev)
    tc = tile_chunks_for(total_words, n)
    utc = unpack_tile_chunks_for(total_words, n, sync=sync is not None)
    ctx.reserve(n)
    stream = torch.cuda.current_stream()

    ev = []

    def step(record):
        if record:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
        ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tc, sync=sync)
        if record:
            e[1].record(stream)
        ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed, chunks_per_tile=utc,
                              sync=sync)
        if record:
            e[2].record(stream)
            ev.append(e)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:  # measurement only: the shards never exchange data
        from capnp_amd import shard
        elapsed = shard.max_over_ranks(elapsed, device=dev)

    # correctness of the timed work (round trip) — outside the timed region
    ok = bool(torch.equal(back, words)) and int((status != 0).sum()) == 0
    P = int(poffs[-1].item())
    U = total_words * 8
    pack_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev)
    unpack_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / len(ev)
    offs_bytes = 8 * (n + 1)
    sync_bytes = 4 * ctx.sync_entries(total_words) if sync is not None else 0
    # algorithmic bytes per launch: words + packed bytes + offsets (+ the
    # record sync index written by pack / read by unpack; + unpack's status
    # and consumed arrays)
    pack_bytes = U + P + 2 * offs_bytes + sync_bytes
    unpack_bytes = P + U + 2 * offs_bytes + 4 * n + 8 * n + sync_bytes
    kernels = {
        "pack": {"ms": round(pack_ms, 4), "alg_bytes": pack_bytes,
                 "GBps": round(pack_bytes / (pack_ms * 1e-3) / 1e9, 1),
                 "unpacked_GiBps": round(U / (pack_ms * 1e-3) / GiB, 2)},
        "unpack": {"ms": round(unpack_ms, 4), "alg_bytes": unpack_bytes,
                   "GBps": round(unpack_bytes / (unpack_ms * 1e-3) / 1e9, 1),
                   "unpacked_GiBps": round(U / (unpack_ms * 1e-3) / GiB, 2)},
    }
    dom = "pack" if pack_ms >= unpack_ms else "unpack"
    achieved = kernels[dom]["GBps"]
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = f"{args.workload}:{n}x{cw}" + (":sync" if sync is not None else "")
        traffic = tj.get(key, {}).get(dom)
    except (OSError, ValueError):
        pass

    e2e = None
    if args.e2e and rank == 0:
        e2e = end_to_end(ctx, torch, words, offs, n, cw, tc, dev)

    ms_per_step = elapsed / args.steps * 1e3
    value = world * U / GiB / (elapsed / args.steps)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 generator, SURVEY §8d)",
            "config": {
                "workload": f"{args.workload}: {n} segments x {cw * 8} B per GPU, "
                            f"{'~30' if args.workload == 'config2' else '~80'} % zero words, "
                            "pack+unpack round trip",
                "segments_per_gpu": n, "segment_bytes": cw * 8,
                "global_unpacked_bytes": world * U, "parallelism": f"shard{world}",
            },
            "roofline": {
                "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
            },
            "kernels": kernels,
            "packed_ratio": round(P / U, 4),
            "sync_index": sync is not None,
            "roundtrip_ok": ok,
        }
        if e2e:
            line["e2e"] = e2e
        if not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def end_to_end(ctx, torch, words, offs, n, cw, tc, dev):
    """Host pinned buffer -> H2D -> pack -> D2H and back (PCIe-bound).
    Reported in DESIGN.md only; never the headline value."""
    from capnp_amd import unpack_tile_chunks_for
    U = n * cw * 8
    h_words = torch.empty(n * cw, dtype=torch.int64, pin_memory=True)
    h_words.copy_(words)
    cap = ctx.batch_bound_bytes(n * cw, n)
    d_words = torch.empty_like(words)
    d_packed = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    h_packed = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    d_back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    h_back = torch.empty(n * cw, dtype=torch.int64, pin_memory=True)
    res = {}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d_words.copy_(h_words, non_blocking=True)
        ctx.pack_batch_into(d_words, offs, d_packed, d_poffs, chunks_per_tile=tc)
        torch.cuda.synchronize()
        P = int(d_poffs[-1].item())
        h_packed[:P].copy_(d_packed[:P], non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        d_packed[:P].copy_(h_packed[:P], non_blocking=True)
        ctx.unpack_batch_into(d_packed, d_poffs, offs, d_back, status,
                              chunks_per_tile=unpack_tile_chunks_for(n * cw, n))
        h_back.copy_(d_back, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = {"encode_GiBps": round(U / (t1 - t0) / GiB, 3),
               "decode_GiBps": round(U / (t2 - t1) / GiB, 3),
               "roundtrip_GiBps": round(U / (t2 - t0) / GiB, 3),
               "note": "pinned host -> H2D -> kernel -> D2H, sequential (no overlap)"}
    assert torch.equal(h_back, h_words)
    # streaming host batch (capnp_stream_*): copy in, kernel and copy out of
    # consecutive slices overlap on three streams
    h_poffs = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
    h_offs = offs.cpu().pin_memory()
    h_status = torch.empty(n, dtype=torch.int32, pin_memory=True)
    slice_words = 4 << 20
    for rep in range(3):
        h_back.zero_()
        t0 = time.perf_counter()
        P = ctx.stream_pack(h_words, h_offs, h_packed, h_poffs, slice_words=slice_words)
        t1 = time.perf_counter()
        ctx.stream_unpack(h_packed, h_poffs, h_offs, h_back, h_status, slice_words=slice_words)
        t2 = time.perf_counter()
        res["stream_encode_GiBps"] = round(U / (t1 - t0) / GiB, 3)
        res["stream_decode_GiBps"] = round(U / (t2 - t1) / GiB, 3)
        res["stream_roundtrip_GiBps"] = round(U / (t2 - t0) / GiB, 3)
    assert torch.equal(h_back, h_words) and int(h_status.sum()) == 0
    res["stream_note"] = (f"capnp_stream_pack_batch / capnp_stream_unpack_batch, "
                          f"{slice_words} words per slice, pinned host buffers")
    return res


if __name__ == "__main__":
    main()
