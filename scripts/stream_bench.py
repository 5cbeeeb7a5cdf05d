#!/usr/bin/env python3
"""Foreign packed stream decode: a ~1 GiB stream of the
reference benchmark's carsales request messages (one segment each,
benchmark/carsales.rs), written by capnp_gpu_write_messages, then read back
with no byte index:
  one_pass   capnp_gpu_read_message_stream (decode once, describe in place)
  two_pass   capnp_gpu_find_messages + capnp_gpu_read_messages (round 2)
GiB/s of unpacked message bytes (tables + segments) over the call's wall
time (blocking calls, device-resident stream).  Prints one JSON line.

    python3 scripts/stream_bench.py [--gib 1.0] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from capnp_amd import Context
    ctx = Context(0)
    total = int(a.gib * (1 << 30)) // 8
    words = torch.empty(total, dtype=torch.int64, device="cuda")
    req = ctx.gen_carsales(words)  # request word offsets (the last may be cut)
    nreq = len(req) - 2  # whole requests only
    req = req[:nreq + 1]
    seg_off = torch.from_numpy(req.astype("int64")).cuda()
    msg_seg = torch.arange(0, nreq + 1, dtype=torch.int64, device="cuda")
    packed, mbo = ctx.write_messages(words, seg_off, msg_seg)
    torch.cuda.synchronize()
    U = int(seg_off[-1].item()) * 8 + 8 * nreq  # segment words + one table word each
    P = packed.numel()
    res = {"workload": f"{nreq} carsales request messages, {U / (1 << 30):.3f} GiB unpacked, "
                       f"{P / (1 << 30):.3f} GiB packed", "messages": nreq,
           "unpacked_bytes": U, "packed_bytes": P}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best, out

    wc = int(U // 8 + 1024)
    t1, out1 = timed(lambda: ctx.decode_stream(packed, words_cap=wc, msgs_cap=nreq + 16,
                                               segs_cap=nreq + 16))
    n1, clean1 = out1[5], out1[6]
    ok1 = n1 == nreq and clean1 and torch.equal(out1[1], mbo)
    res["one_pass"] = {"s": round(t1, 5), "GiBps": round(U / t1 / (1 << 30), 2), "ok": bool(ok1)}

    def two_pass():
        offs, n = ctx.find_messages(packed, max_msgs=nreq + 16)
        return ctx.read_messages(packed, offs, words_cap=wc, segs_cap=nreq + 16), n

    t2, out2 = timed(two_pass)
    res["two_pass"] = {"s": round(t2, 5), "GiBps": round(U / t2 / (1 << 30), 2),
                       "ok": bool(out2[1] == nreq)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
