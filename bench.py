#!/usr/bin/env python3
"""Benchmark: packed encode+decode of device-resident Cap'n Proto segments.

Workloads (--workload; SURVEY.md §8d, BASELINE.json configs):
  config2   (default, configs[1]) 1 Mi segments x 1 KiB per GPU, ~30 % zero
            words (seeded splitmix64 generator)
  config3   the same shape at >= 80 % zero words (configs[2]; --chunks
            23400000 for the 4 GiB-packed size)
  carsales  1 Mi x 1 KiB carsales-shaped segments: the reference benchmark's
            request stream (benchmark/carsales.rs:84-150 on FastRand,
            common.rs:22-70) cut into 128-word chunks (north_star workload)
  config4   mixed 64 B - 64 KiB segments, ~1 GiB (configs[3])
  config5   8 Mi x 1 KiB per GPU = 8 GiB (configs[4]: 64 GiB over 8 GPUs)
One step = PACK the whole batch (capnp_gpu_pack_batch_sync) and UNPACK it
back (capnp_gpu_unpack_batch_sync): the encode+decode round trip of the
metric.  value = unpacked GiB per step (all ranks) / step time.

Multi-GPU: `--gpus N` (N > 1) started as a plain process re-launches itself
under torch.distributed.run with N ranks (a child process, before any GPU
call); one process per GPU, each rank packs and unpacks its own shard of
independent segments, no data-path collective; scaling is weak.  The
collectives are the barrier and the max-over-ranks of the timing only.

The JSON line also carries
  roofline      the dominant kernel's algorithmic bytes per launch / its mean
                launch time (HIP events on the launch stream) vs 8 TB/s;
  cpu_baseline  the reference's CPU codec loops (oracle/refloop_oracle.c, a C
                restatement; the reference is Rust and cannot be built here)
                timed on a bounded sample of the same workload on this host.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MEASURED_COPY_GBS = 6290.0  # measured float4 copy (same source)
PZ = {"config2": 1288490189, "config3": 3435973837, "config5": 1288490189,
      "config4": 1288490189}
METRIC = "GiB/s packed encode+decode, device-resident segments; % HBM roofline"
GiB = float(1 << 30)
CARSALES_RANK_STRIDE = 100_000  # rank r's requests start at r x this (~90 k per GiB)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed load before the warm-up steps: the GPU's clocks run "
                         "~10 %% slow for the first ~30 ms of load after idle "
                         "(profiles/r04g_clock_curve.txt); 0 = off")
    ap.add_argument("--chunks", type=int, default=0,
                    help="segments per GPU (0 = the workload's size)")
    ap.add_argument("--chunk-words", type=int, default=128)
    ap.add_argument("--workload", default="config2",
                    choices=["config2", "config3", "carsales", "config4", "config5"])
    ap.add_argument("--cpu-sample-words", type=int, default=1 << 25)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time host->device->host")
    ap.add_argument("--no-sync", action="store_true",
                    help="pack without the record sync index; unpack walks whole chunks")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous / reporting only, no GPU (gloo; tests)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """--gpus N from a plain process: run this script under
    torch.distributed.run with N ranks as a child process (nothing here has
    touched the GPU) and exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None
    when unlimited / not readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def cpu_share():
    """What this process may run on: the affinity mask (the threads actually
    usable), the cgroup quota and OMP_NUM_THREADS, each as found."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    env = os.environ.get("OMP_NUM_THREADS")
    return {"affinity_cpus": aff, "cgroup_quota_cpus": _cgroup_cpus(),
            "omp_num_threads": int(env) if env and env.isdigit() else None,
            "host_cpus": os.cpu_count()}


def cpu_threads(args):
    """Threads for the CPU baseline: the affinity mask's CPU count
    (len(os.sched_getaffinity(0))), capped by the cgroup quota and by
    OMP_NUM_THREADS when either is set (the GPU pool grants each box a
    16-CPU share of a larger host; all three are reported)."""
    if args.cpu_threads:
        return args.cpu_threads
    sh = cpu_share()
    n = sh["affinity_cpus"] or sh["host_cpus"] or 1
    for cap in (sh["cgroup_quota_cpus"], sh["omp_num_threads"]):
        if cap:
            n = min(n, cap)
    return max(1, n)


def config1_baseline(threads, target_words=1 << 25, reps=3):
    """BASELINE configs[0], `benchmark carsales bytes reuse packed`
    (benchmark/benchmark.rs:207-259, carsales.rs:140-150): the codec calls of
    each iteration, serialize_packed::write_message + read_message of one
    carsales request, on the CPU oracle (the C restatement of the reference
    codec; there is no Rust toolchain to run the reference itself).  The
    requests are the benchmark's own FastRand chain (oracle/carsales_oracle.c);
    one request per task on `threads` threads, and on one thread."""
    import numpy as np
    import oracle_lib as O
    words, msg_off, _ = O.carsales_stream(target_words)
    m = len(msg_off) - 2  # requests complete in the sample
    mo = msg_off[:m + 1]
    ww = words[:int(mo[-1])]
    um = 8 * len(ww)
    runs = [O.refloop_messages_roundtrip_mt(ww, mo, threads) for _ in range(reps)]
    assert all(r[3] for r in runs)
    bm = min(runs, key=lambda r: r[0] + r[1])
    m1 = max(1, m // 16)
    b1 = min((O.refloop_messages_roundtrip_mt(words[:int(msg_off[m1])], msg_off[:m1 + 1], 1)
              for _ in range(2)), key=lambda r: r[0] + r[1])
    u1 = 8 * int(msg_off[m1])
    # the parity oracle's branchy loops on the same requests (the round-3 figure)
    ro = min((O.messages_roundtrip_mt(ww, mo, threads) for _ in range(2)),
             key=lambda r: r[0] + r[1])
    assert ro[3] and ro[2] == bm[2]
    return {
        "workload": "config1: benchmark carsales bytes reuse packed, codec calls "
                    "(write_message + read_message per request)",
        "requests": int(m), "unpacked_bytes": um, "packed_ratio": round(bm[2] / um, 4),
        "threads": threads,
        "roundtrip_gibps": round(um / (bm[0] + bm[1]) / GiB, 3),
        "write_gibps": round(um / bm[0] / GiB, 3), "read_gibps": round(um / bm[1] / GiB, 3),
        "requests_per_s": round(m / (bm[0] + bm[1]), 1),
        "single_thread_roundtrip_gibps": round(u1 / (b1[0] + b1[1]) / GiB, 3),
        "single_thread_requests_per_s": round(m1 / (b1[0] + b1[1]), 1),
        "oracle_roundtrip_gibps": round(um / (ro[0] + ro[1]) / GiB, 3),
        "kind": "port",
        "note": f"best of {reps}; {m} requests ({um / GiB:.3f} GiB) of the reference "
                f"benchmark's chain, the reference's loops (oracle/refloop_oracle.c; "
                f"read_message zeroes the body as allocate_zeroed_vec does); single "
                f"thread on the first {m1}; oracle_roundtrip_gibps: the parity oracle's "
                f"branchy loops",
    }


def cpu_baseline(args, threads):
    """The CPU oracle on a bounded sample of the same workload on this host:
    chunk-level pack + unpack (all workloads), and for carsales the
    reference benchmark's per-request write_message + read_message."""
    import numpy as np
    import oracle_lib as O
    cw = args.chunk_words
    n = max(1, args.cpu_sample_words // cw)
    offs = np.arange(0, (n + 1) * cw, cw, dtype=np.uint64)
    if args.workload == "carsales":
        words, msg_off, _ = O.carsales_stream(n * cw)
    elif args.workload == "config4":
        # the first segments of rank 0's config-4 batch (same sizes, kinds and
        # generator as the GPU workload) up to the sample's words
        sizes, kinds = config4_layout(0)
        n = max(1, int(np.searchsorted(np.cumsum(sizes), args.cpu_sample_words, side="right")))
        offs = np.concatenate([[0], np.cumsum(sizes[:n])]).astype(np.uint64)
        words = O.gen_fill(offs, kinds=kinds[:n], pz=PZ["config4"], id0=0)
    else:
        words = O.gen_fill(offs, kind0=0, pz=PZ.get(args.workload, PZ["config2"]))

    def timed(nn, thr, reps):
        """The reference's loops (oracle/refloop_oracle.c): buffers allocated
        and mapped before the clock, bytes checked against the parity oracle
        after it."""
        o = offs[:nn + 1]
        w = words[:int(o[-1])]
        b = O.RefloopBatch(w, o, thr)
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            st = b.pack()
            t1 = time.perf_counter()
            b.unpack()
            t2 = time.perf_counter()
            assert st == 0 and (b.status == 0).all() and np.array_equal(b.back[:len(w)], w)
            if best is None or t2 - t0 < best[0]:
                best = (t2 - t0, t1 - t0, t2 - t1)
        stream, soffs = b.packed_stream()
        st, ref, ref_offs = O.pack_batch(w, o)
        assert st == 0 and np.array_equal(stream, ref) and np.array_equal(soffs, ref_offs)
        return best

    def timed_oracle(nn, thr, reps):
        """The parity oracle's branchy loops (round 3's baseline), same sample."""
        o = offs[:nn + 1]
        w = words[:int(o[-1])]
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            st, packed, poffs = O.pack_batch(w, o, threads=thr)
            back, status, _ = O.unpack_batch(packed, poffs, o, threads=thr)
            t1 = time.perf_counter()
            assert st == 0 and (status == 0).all() and np.array_equal(back, w)
            best = t1 - t0 if best is None else min(best, t1 - t0)
        return best

    best = timed(n, threads, args.cpu_reps)
    n1 = max(1, n // 16)
    one = timed(n1, 1, 2)
    u, u1 = int(offs[n]) * 8, int(offs[n1]) * 8
    orc = timed_oracle(n, threads, 2)
    orc1 = timed_oracle(n1, 1, 1)
    shape = (f"{n} segments of 64 B - 64 KiB" if args.workload == "config4"
             else f"{n} segments x {cw * 8} B")
    share = cpu_share()
    res = {
        "value": round(u / best[0] / GiB, 3),
        "unit": "GiB/s",
        "cores": threads,
        **share,
        "kind": "port",
        "sample": f"{shape} ({u / GiB:.3f} GiB) of the same workload, "
                  f"pack+unpack per segment, best of {args.cpu_reps}, {threads} threads, "
                  f"the reference's branch-free loops (oracle/refloop_oracle.c, gcc -O3: "
                  f"serialize_packed.rs:304-439 / :80-228, outputs mapped before timing, "
                  f"bytes checked against the parity oracle); cores = threads used = the "
                  f"affinity mask's CPUs capped by the cgroup quota and OMP_NUM_THREADS",
        "pack_gibps": round(u / best[1] / GiB, 3),
        "unpack_gibps": round(u / best[2] / GiB, 3),
        "single_thread_gibps": round(u1 / one[0] / GiB, 3),
        "single_thread_pack_gibps": round(u1 / one[1] / GiB, 3),
        "single_thread_unpack_gibps": round(u1 / one[2] / GiB, 3),
        # round 3's baseline: the parity oracle (oracle/packed_oracle.c), branchy loops
        "oracle_gibps": round(u / orc / GiB, 3),
        "oracle_single_thread_gibps": round(u1 / orc1 / GiB, 3),
    }
    # BASELINE configs[0] rides on every line (the driver runs the default
    # workload only)
    res["config1"] = config1_baseline(threads, reps=args.cpu_reps)
    return res


def config4_layout(rank):
    """Config 4's segment sizes (words, log-uniform 8 .. 8192) and generator
    kinds (0: ~30 %-zero words, 1: long zero runs, 2: long literal runs) for
    one rank: ~1 GiB of words."""
    import numpy as np
    rng = np.random.default_rng(4 + rank)
    target = (1 << 30) // 8
    sizes, total = [], 0
    while total < target:
        s = int(np.exp(rng.uniform(np.log(8), np.log(8193))))
        sizes.append(s)
        total += s
    kinds = rng.choice(3, size=len(sizes), p=[0.8, 0.1, 0.1]).astype(np.uint8)
    return np.array(sizes, np.int64), kinds


def make_workload(args, ctx, torch, dev, rank):
    """-> (words, chunk_word_off, n, description) resident in HBM."""
    import numpy as np
    cw = args.chunk_words
    wl = args.workload
    if wl == "config4":
        sizes, kinds = config4_layout(rank)
        n, total = len(sizes), int(sizes.sum())
        offs_h = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        offs = torch.from_numpy(offs_h).to(dev)
        words = torch.empty(total, dtype=torch.int64, device=dev)
        ctx.gen_batch(words, offs, pz_thresh=PZ[wl], kinds=torch.from_numpy(kinds).to(dev),
                      id0=rank * 10_000_000)
        return words, offs, n, (f"config4: {n} segments, 64 B - 64 KiB log-uniform, "
                                f"{8 * total / GiB:.3f} GiB per GPU (80 % ~30 %-zero words, "
                                "10 % long zero runs, 10 % long literal runs)")
    n = args.chunks or {"config5": 8 << 20}.get(wl, 1 << 20)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device=dev)
    words = torch.empty(n * cw, dtype=torch.int64, device=dev)
    if wl == "carsales":
        req = ctx.gen_carsales(words, skip_requests=rank * CARSALES_RANK_STRIDE)
        desc = (f"carsales: {n} segments x {cw * 8} B per GPU cut from {len(req) - 1} "
                f"carsales requests (benchmark/carsales.rs, FastRand chain from request "
                f"{rank * CARSALES_RANK_STRIDE})")
    else:
        ctx.gen_batch(words, offs, pz_thresh=PZ[wl], id0=rank * n)
        desc = (f"{wl}: {n} segments x {cw * 8} B per GPU, "
                f"{'~80' if wl == 'config3' else '~30'} % zero words")
    return words, offs, n, desc


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    if args.dry_run:
        return dry_run(args, world)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a process group whenever a launcher started this rank (torchrun sets
    # the rendezvous variables even at one rank), so the barrier /
    # max-over-ranks path the 8-GPU run takes is one a one-GPU box exercises
    dist_on = world > 1 or all(k in os.environ for k in
                               ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"))
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from capnp_amd import Context, tile_chunks_for, unpack_tile_chunks_for
    ctx = Context(local)
    words, offs, n, desc = make_workload(args, ctx, torch, dev, rank)
    total_words = words.numel()
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

    # Settle: untimed steps until the GPU has been under load for
    # --settle-ms (at most 400 steps), so the timed steps see the steady
    # clocks a continuously running codec sees, not the power-management
    # transient after idle (per-step kernel times 530-590 us for the first
    # ~10 steps, 455-465 us after ~30 ms: scripts/clock_curve.py).  Then
    # the W warm-up steps, then exactly K timed steps.
    settle_steps, settle_t0 = 0, time.perf_counter()
    while args.settle_ms > 0 and settle_steps < 400:
        for _ in range(8):
            step(False)
        settle_steps += 8
        torch.cuda.synchronize()
        if (time.perf_counter() - settle_t0) * 1e3 >= args.settle_ms:
            break
    settle_ms = (time.perf_counter() - settle_t0) * 1e3
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:  # measurement only: the shards never exchange data
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

    def kern(ms, nbytes):
        return {"ms": round(ms, 4), "alg_bytes": nbytes,
                "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "unpacked_GiBps": round(U / (ms * 1e-3) / GiB, 2)}

    kernels = {"pack": kern(pack_ms, pack_bytes), "unpack": kern(unpack_ms, unpack_bytes)}
    if sync is not None:
        # the reference-compatible decode (a stream with no side-band index),
        # timed after the headline loop on the same packed batch
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = max(3, args.steps // 4)
        t_s = time.perf_counter()  # (settle again: the checks above left the GPU idle)
        while True:
            for _ in range(4):
                ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed,
                                      chunks_per_tile=unpack_tile_chunks_for(total_words, n))
            torch.cuda.synchronize()
            if args.settle_ms <= 0 or (time.perf_counter() - t_s) * 1e3 >= args.settle_ms / 2:
                break
        e[0].record(stream)
        for _ in range(reps):
            ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed,
                                  chunks_per_tile=unpack_tile_chunks_for(total_words, n))
        e[1].record(stream)
        torch.cuda.synchronize()
        ok_ns = bool(torch.equal(back, words)) and int((status != 0).sum()) == 0
        kernels["unpack_nosync"] = kern(e[0].elapsed_time(e[1]) / reps,
                                        P + U + 2 * offs_bytes + 12 * n)
        kernels["unpack_nosync"]["roundtrip_ok"] = ok_ns
        ok = ok and ok_ns
        # and the index-free pack (the same bytes, no sync index written)
        e[0].record(stream)
        for _ in range(reps):
            ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=tc)
        e[1].record(stream)
        torch.cuda.synchronize()
        ok = ok and int(poffs[-1].item()) == P
        kernels["pack_nosync"] = kern(e[0].elapsed_time(e[1]) / reps, U + P + 2 * offs_bytes)
    dom = "pack" if pack_ms >= unpack_ms else "unpack"
    achieved = kernels[dom]["GBps"]
    traffic = traffic_rw = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = f"{args.workload}:{n}x{args.chunk_words}" + (":sync" if sync is not None else "")
        ent = tj.get(key, {}).get(dom)
        if isinstance(ent, dict):  # per-kernel HBM bytes per launch, read / write split
            traffic = ent["total"]
            traffic_rw = {"read": ent["read"], "write": ent["write"],
                          "source": "profiles/traffic.json (rocprofv3 FETCH_SIZE x 2, WRITE_SIZE)"}
    except (OSError, ValueError, KeyError):
        pass

    e2e = None
    if args.e2e and rank == 0:
        e2e = end_to_end(ctx, torch, words, offs, n, tc, dev)

    ms_per_step = elapsed / args.steps * 1e3
    value = world * U / GiB / (elapsed / args.steps)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "process_group": dist.get_backend() if dist_on else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"steps": settle_steps, "ms": round(settle_ms, 1),
                       "why": "untimed load before the warm-up steps: clocks settle after "
                              "~30 ms of load (DESIGN.md, Measurement)"},
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic: the reference benchmark's carsales requests (FastRand chain)"
                     if args.workload == "carsales" else
                     "synthetic (seeded splitmix64 generator, SURVEY §8d)"),
            "config": {
                "workload": desc + ", pack+unpack round trip",
                "segments_per_gpu": n, "unpacked_bytes_per_gpu": U,
                "global_unpacked_bytes": world * U, "parallelism": f"shard{world}",
            },
            "roofline": {
                "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_rw": traffic_rw,
            },
            "roundtrip_frac_of_hbm": round((pack_bytes + unpack_bytes) /
                                           ((pack_ms + unpack_ms) * 1e-3) / 1e9 /
                                           HBM_PEAK_GBS, 4),
            "aggregate_frac_of_hbm": round(world * (pack_bytes + unpack_bytes) /
                                           (elapsed / args.steps) / 1e9 /
                                           (world * HBM_PEAK_GBS), 4),
            "kernels": kernels,
            # reference-compatible round trip: no side-band index either way,
            # U / (pack without index + index-free unpack), kernel times
            "roundtrip_noindex_GiBps": (
                round(U / GiB / ((kernels["pack_nosync"]["ms"] +
                                  kernels["unpack_nosync"]["ms"]) * 1e-3), 2)
                if "unpack_nosync" in kernels else None),
            "packed_ratio": round(P / U, 4),
            "sync_index": sync is not None,
            "roundtrip_ok": ok,
        }
        if e2e:
            line["e2e"] = e2e
        if not args.no_cpu and world == 1:  # (the CPU baseline is an N=1 figure)
            line["cpu_baseline"] = cpu_baseline(args, cpu_threads(args))
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def dry_run(args, world):
    """The launcher path without a GPU: each rank joins a gloo group, the
    max over ranks of a per-rank stand-in time is taken, rank 0 reports."""
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from capnp_amd import shard
        elapsed = shard.max_over_ranks(0.01 * (rank + 1))
        dist.barrier()
        dist.destroy_process_group()
    else:
        elapsed = 0.01
    print(json.dumps({"dry_run": True, "rank": rank, "world": world}), file=sys.stderr,
          flush=True)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world,
                          "dry_run": True, "max_elapsed": elapsed, "steps": args.steps,
                          "warmup": args.warmup}), flush=True)


def end_to_end(ctx, torch, words, offs, n, tc, dev):
    """Host pinned buffer -> H2D -> pack -> D2H and back (PCIe-bound).
    Reported in DESIGN.md only; never the headline value."""
    from capnp_amd import unpack_tile_chunks_for
    total = words.numel()
    U = total * 8
    h_words = torch.empty(total, dtype=torch.int64, pin_memory=True)
    h_words.copy_(words)
    cap = ctx.batch_bound_bytes(total, n)
    d_words = torch.empty_like(words)
    d_packed = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    h_packed = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    d_back = torch.empty_like(words)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    h_back = torch.empty(total, dtype=torch.int64, pin_memory=True)
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
                              chunks_per_tile=unpack_tile_chunks_for(total, n))
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
        ctx.stream_pack(h_words, h_offs, h_packed, h_poffs, slice_words=slice_words)
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
