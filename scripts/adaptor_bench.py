#!/usr/bin/env python3
"""Throughput of the streaming adaptors (capnp-futures PackedRead /
PackedWrite equivalents, csrc/stream_io.hip) over an in-memory inner
stream, in 1 MiB calls: GiB/s of unpacked bytes.  The
packed stream is config 2's data (30 % zero words), 256 MiB unpacked.
Prints one JSON line.  (Calls pass views of the caller's buffers, as the
reference's poll_write(&[u8]) / poll_read(&mut [u8]) do: no per-call copy
in the harness.)

    python3 scripts/adaptor_bench.py [--mib 256] [--call-mib 1] [--lib path]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


class MemRead:
    def __init__(self, data):
        self.m = memoryview(data)
        self.pos = 0

    def read(self, n):
        r = self.m[self.pos:self.pos + n]
        self.pos += len(r)
        return r


class MemWrite:
    """A file-like sink over one preallocated buffer (a socket or file
    buffer): each write copies into it, no allocation per call."""

    def __init__(self, cap):
        self.buf = bytearray(cap)
        self.mv = memoryview(self.buf)
        self.n = 0

    def write(self, b):
        k = len(b)
        self.mv[self.n:self.n + k] = b
        self.n += k
        return k

    def value(self):
        return self.buf[:self.n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="also time the reference's loops")
    ap.add_argument("--call-mib", type=float, default=1.0)
    ap.add_argument("--lib", default="", help="another build of the library (A/B)")
    a = ap.parse_args()
    if a.lib:
        os.environ["CAPNP_PACKED_LIB"] = a.lib
    import torch
    from capnp_amd import Context, serialize_packed_async as spa
    ctx = Context(0)
    nw = a.mib << 17
    cw = 128
    offs = torch.arange(0, nw + 1, cw, dtype=torch.int64, device="cuda")
    words = torch.empty(nw, dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=1288490189)
    raw = words.cpu().numpy().tobytes()
    call = int(a.call_mib * (1 << 20))
    warm = min(len(raw) // 8, 16 << 20) // call * call  # untimed lead-in of each adaptor
    # write: 1 MiB calls of unpacked bytes (views of the caller's buffer, as
    # a Rust caller passes &[u8]), then flush.  The first `warm` bytes go
    # untimed: an adaptor's first calls create its background context and
    # staging buffers (the reader's first unit took 26 ms on the box).
    mv = memoryview(raw)
    GiB = float(1 << 30)
    for run in range(a.runs):
        sink = MemWrite(len(raw) + len(raw) // 8 + (1 << 20))
        w = spa.PackedWrite(sink, ctx=ctx, inner_copies=True)  # (MemWrite copies)
        for i in range(0, warm, call):
            w.write_all(mv[i:i + call])
        t0 = time.perf_counter()
        for i in range(warm, len(raw), call):
            w.write_all(mv[i:i + call])
        w.flush_blocking()
        tw = time.perf_counter() - t0
        del w
        packed = bytes(sink.value())
        # read: calls of up to 1 MiB into the caller's buffer (poll_read(&mut
        # [u8]) -> readinto) until the end, the first `warm` bytes untimed
        r = spa.PackedRead(MemRead(packed), ctx=ctx, readahead=True)  # (a memory source: bulk)
        got = bytearray(len(raw) + call)
        gv = memoryview(got)
        pos = 0
        while pos < warm:
            k = r.readinto(gv[pos:pos + min(call, warm - pos)])
            if not k:
                break
            pos += k
        p0 = pos
        t0 = time.perf_counter()
        while True:
            k = r.readinto(gv[pos:pos + call])
            if not k:
                break
            pos += k
        tr = time.perf_counter() - t0
        del r
        ok = pos == len(raw) and gv[:pos] == raw
        print(json.dumps({
            "run": run,
            "workload": f"config-2 data, {len(raw) / GiB:.3f} GiB unpacked, {len(packed) / GiB:.3f} GiB "
                        f"packed, {call} B calls, in-memory inner stream (preallocated sink)",
            "timed_bytes": {"write": len(raw) - warm, "read": len(raw) - p0, "untimed_lead_in": warm},
            "write_GiBps": round((len(raw) - warm) / GiB / tw, 3),
            "read_GiBps": round((len(raw) - p0) / GiB / tr, 3),
            "write_s": round(tw, 4), "read_s": round(tr, 4), "ok": ok}), flush=True)
    if a.cpu:
        # the reference's loops on the same bytes: one stream on one thread
        # (a PackedWrite / PackedRead is serial), and the stream cut at the
        # call size on 16 threads (independent write_all / read units)
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        wn = np.frombuffer(raw, np.uint64)
        sample = wn[:min(len(wn), 32 << 20)]  # (256 MiB: a bounded CPU sample)
        for threads in (1, 16):
            offs = np.arange(0, len(sample) + 1, call // 8, dtype=np.uint64)
            if offs[-1] != len(sample):
                offs = np.append(offs, np.uint64(len(sample)))
            best = None
            for _ in range(2):
                t_w, t_r, pb, okc = O.refloop_messages_roundtrip_mt(sample, offs, threads)
                assert okc
                best = (t_w, t_r) if best is None else (min(best[0], t_w), min(best[1], t_r))
            print(json.dumps({"cpu_reference_loops": {
                "threads": threads, "sample_GiB": round(len(sample) * 8 / GiB, 3),
                "write_GiBps": round(len(sample) * 8 / GiB / best[0], 3),
                "read_GiBps": round(len(sample) * 8 / GiB / best[1], 3)}}), flush=True)


if __name__ == "__main__":
    main()
