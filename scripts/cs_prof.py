#!/usr/bin/env python3
"""Per-tile phase timeline of pack_cs_kernel from the PACK_PROF=3 build
(`make -C capnproto-rust_amd variant FILE=pack NAME=prof3 DEFS=-DPACK_PROF=3`): start, loads landed, pass 1 +
publish, pass 2, look-back, end (s_memrealtime, 100 MHz).  Prints the mean of
each phase and how many tiles are in each phase on average over the launch
(the memory-level parallelism of the load phase).  Diagnostic only.

    python3 scripts/cs_prof.py [--chunks N] [--pz P] [--iters K]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--pz", type=int, default=1288490189)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--lib", default="")
    ap.add_argument("--pipe", action="store_true",
                    help="pack_pipe_kernel's trace layout (CAPNP_PACK_PIPE on)")
    a = ap.parse_args()
    import torch
    from capnp_amd import Context
    path = a.lib or os.path.join(ROOT, "capnproto-rust_amd/build/abl/libcapnp_packed_prof3.so")
    L = C.CDLL(path)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
    L.capnp_ctx_create.restype = vp
    L.capnp_gpu_pack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
    L.capnp_gpu_pack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, u32, vp]
    L.capnp_ctx_reserve.argtypes = [vp, sz]
    L.capnp_pack_trace.argtypes = [vp]
    st = C.c_int(0)
    h = vp(L.capnp_ctx_create(0, C.byref(st)))
    n, cw, tc = a.chunks, 128, 16
    ctx = Context(0)
    offs = torch.arange(0, (n + 1) * cw, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(n * cw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=a.pz)
    ref_out, ref_oo = ctx.pack_batch(words, offs)
    cap = ctx.batch_bound_bytes(n * cw, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sync = torch.empty(ctx.sync_entries(n * cw), dtype=torch.int32, device="cuda")
    L.capnp_ctx_reserve(h, n)
    ntiles = (n + tc - 1) // tc
    trace = torch.zeros(ntiles * 8, dtype=torch.int64, device="cuda")
    L.capnp_pack_trace(C.c_void_p(trace.data_ptr()))
    stream = torch.cuda.current_stream()
    P = C.c_void_p
    for it in range(a.iters + 1):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if a.sync:
            L.capnp_gpu_pack_batch_sync_tuned(h, P(words.data_ptr()), P(offs.data_ptr()), n,
                                              P(out.data_ptr()), cap, P(oo.data_ptr()),
                                              P(sync.data_ptr()), tc, P(stream.cuda_stream))
        else:
            L.capnp_gpu_pack_batch_tuned(h, P(words.data_ptr()), P(offs.data_ptr()), n,
                                         P(out.data_ptr()), cap, P(oo.data_ptr()), tc,
                                         P(stream.cuda_stream))
        e1.record(stream)
        e1.synchronize()
        if it == 0:
            continue
        ok = torch.equal(oo, ref_oo) and torch.equal(out[:ref_out.numel()], ref_out)
        T = trace.view(ntiles, 8).cpu().numpy().astype(np.int64)
        t0 = T[:, 0].min()
        span = (T[:, 5].max() - t0) / 100.0
        if a.pipe:
            # [6] iteration start, [0] wave 0's pass 1 done, [1] published, [2] pass 2 done,
            # [3] look-back start (next iteration), [4] offset known, [5] copied out
            order = [6, 0, 1, 2, 3, 4, 5]
            ph = ["words+pass1(w0)", "barrier+pub", "retire-prev+pass2", "next-pass1", "lookback",
                  "copyout"]
            t0 = T[:, 6].min()
            span = (T[:, 5].max() - t0) / 100.0
        else:
            order = [0, 1, 2, 3, 4, 5]
            ph = ["load", "pass1+pub", "pass2", "lookback", "copyout"]
        means = [(T[:, order[k + 1]] - T[:, order[k]]).mean() / 100.0 for k in range(len(ph))]
        life = (T[:, 5] - T[:, order[0]]).mean() / 100.0
        # average tiles in each phase over the launch = sum of durations / span
        inflight = [(T[:, order[k + 1]] - T[:, order[k]]).sum() / 100.0 / span
                    for k in range(len(ph))]
        starts = np.sort(T[:, order[0]] - t0) / 100.0
        print(f"iter {it}: {e0.elapsed_time(e1) * 1e3:.1f} us (traced span {span:.1f}) ok={ok} "
              f"tiles={ntiles} lifetime {life:.2f} us")
        print("   phase us : " + "  ".join(f"{p} {m:.2f}" for p, m in zip(ph, means)))
        print("   in flight: " + "  ".join(f"{p} {x:.0f}" for p, x in zip(ph, inflight))
              + f"  (total {sum(inflight):.0f})")
        ok7 = (T[:, 7] >= T[:, 3]) & (T[:, 7] <= T[:, 4]) & (T[:, 7] > 0)
        if not a.pipe and ok7.mean() > 0.9:  # look-back split: own group, then groups
            w = (T[ok7, 7] - T[ok7, 3]) / 100.0
            g = (T[ok7, 4] - T[ok7, 7]) / 100.0
            print(f"   lookback: own group {w.mean():.2f} (p90 {np.percentile(w, 90):.2f})  "
                  f"group records {g.mean():.2f} (p90 {np.percentile(g, 90):.2f}) us "
                  f"({ok7.sum()} tiles)")
            lb = (T[:, 4] - T[:, 3]) / 100.0
            r = np.arange(ntiles) % 64
            print("   lookback by tile in group (r 0, 1-15, 16-47, 48-62, 63): " + "  ".join(
                f"{lb[m].mean():.2f}" for m in (r == 0, (r >= 1) & (r < 16), (r >= 16) & (r < 48),
                                                (r >= 48) & (r < 63), r == 63)))
        if not a.pipe:
            xcc = (T[:, 6] >> 32) & 0xF
            same = (xcc[1:] == xcc[:-1]).mean()
            b8 = (xcc == (np.arange(ntiles) % 8)).mean()
            print(f"   XCD: tile t and t+1 on the same XCD {same:.3f}; XCD == t % 8 for {b8:.3f}")
            # how far a tile's start trails its predecessor's publish (pass 1 done)
            gap = (T[1:, 2] - T[:-1, 2]) / 100.0
            print(f"   publish(t) - publish(t-1): mean {gap.mean():.2f} p10/p90 "
                  f"{np.percentile(gap, 10):.2f}/{np.percentile(gap, 90):.2f} us")
            # the earliest a tile's offset can be known: every earlier tile has
            # published its aggregate (cummax of the publish times before t);
            # what the look-back waits beyond that is the chain's own latency
            ready = np.maximum.accumulate(T[:, 2])
            ready = np.concatenate([[T[0, 2]], ready[:-1]])
            inh = np.maximum(0, ready - T[:, 3]) / 100.0
            lb = (T[:, 4] - T[:, 3]) / 100.0
            extra = (T[:, 4] - np.maximum(ready, T[:, 3])) / 100.0
            print(f"   lookback {lb.mean():.2f}: predecessors unpublished at its start {inh.mean():.2f} "
                  f"(p90 {np.percentile(inh, 90):.2f}; {(inh > 0).mean():.3f} of tiles), "
                  f"beyond the last publish {extra.mean():.2f} (p90 {np.percentile(extra, 90):.2f}) us")
            # dispatch skew by XCD: mean start time of each XCD's tiles relative
            # to the tile-index order (start - the linear fit of start vs t)
            st = (T[:, 0] - t0) / 100.0
            fit = np.polyval(np.polyfit(np.arange(ntiles), st, 1), np.arange(ntiles))
            print("   start - fit by XCD: " + " ".join(
                f"{(st - fit)[xcc == x].mean():+.2f}" for x in range(8)))
            pub = (T[:, 2] - t0) / 100.0
            late = pub - np.minimum.accumulate(pub[::-1])[::-1]
            print(f"   publish later than some later tile's: mean {late.mean():.2f} "
                  f"p90 {np.percentile(late, 90):.2f} us")
        q = np.percentile(T[:, 5] - T[:, order[0]], [10, 50, 90]) / 100.0
        print(f"   lifetime p10/p50/p90 {q[0]:.2f}/{q[1]:.2f}/{q[2]:.2f} us; "
              f"first start->last start {starts[-1] - starts[0]:.1f} us")


if __name__ == "__main__":
    main()
