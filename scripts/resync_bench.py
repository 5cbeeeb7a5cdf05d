"""Times the index-free decode (capnp_gpu_unpack_batch_resync) against the
serial-walk batch unpack (capnp_gpu_unpack_batch, no index) on the same packed
batches, and checks both round trips.  Host-timed (the resync call blocks).

usage: python scripts/resync_bench.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from capnp_amd import Context  # noqa: E402

PZ30 = 1288490189


def workload(ctx, name):
    rng = np.random.default_rng(7)
    if name == "config4_1GiB":
        sizes = np.exp(rng.uniform(np.log(8), np.log(8192), 200000)).astype(np.int64)
        kinds = rng.choice([0, 1, 2], len(sizes), p=[0.8, 0.1, 0.1]).astype(np.uint8)
        keep = np.cumsum(sizes) <= (1 << 27)
        sizes, kinds = sizes[keep], kinds[keep]
    elif name.startswith("config4k"):  # config4k<K>_1GiB: config 4's sizes, every segment kind K
        sizes = np.exp(rng.uniform(np.log(8), np.log(8192), 200000)).astype(np.int64)
        keep = np.cumsum(sizes) <= (1 << 27)
        sizes = sizes[keep]
        kinds = np.full(len(sizes), int(name[len("config4k")]), np.uint8)
    elif name == "config2_1GiB":
        sizes = np.full(1 << 20, 128, np.int64)
        kinds = np.zeros(len(sizes), np.uint8)
    elif name.startswith("one_chunk_"):
        mib = int(name.split("_")[2][:-3])
        sizes = np.array([mib << 17], np.int64)
        kinds = np.zeros(1, np.uint8)
    else:
        raise ValueError(name)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(sizes)])).cuda()
    words = torch.empty(int(offs[-1]), dtype=torch.int64, device="cuda")
    ctx.gen_batch(words, offs, pz_thresh=PZ30, kinds=torch.from_numpy(kinds).cuda(), id0=11)
    packed, poffs = ctx.pack_batch(words, offs)
    torch.cuda.synchronize()
    return words, offs, packed, poffs


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--serial-max-mib", type=int, default=64,
                    help="skip the serial unpack of single chunks above this size")
    ap.add_argument("--corrupt", action="store_true",
                    help="also time the batch with one chunk that fails its check "
                         "(its word count one too many)")
    ap.add_argument("--workloads", default="config2_1GiB,config4_1GiB,one_chunk_16MiB,"
                                            "one_chunk_256MiB")
    a = ap.parse_args()
    ctx = Context(0)
    for name in a.workloads.split(","):
        words, offs, packed, poffs = workload(ctx, name)
        n = offs.numel() - 1
        ub = words.numel() * 8
        back = torch.zeros_like(words)
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        info = {}

        def rs():
            info["r"] = ctx.unpack_batch_resync_into(packed, poffs, offs, back, st)

        t_rs = timed(rs, a.reps)
        ok_rs = bool(torch.equal(back, words)) and bool((st == 0).all().item())
        rec = {"workload": name, "chunks": n, "unpacked_bytes": ub,
               "packed_bytes": int(packed.numel()), "resync_ms": round(t_rs * 1e3, 3),
               "resync_GiBps": round(ub / t_rs / 2**30, 1), "resync_ok": ok_rs,
               "passes": info["r"][0], "serial_fallback": info["r"][1]}
        if not (name.startswith("one_chunk_") and ub > a.serial_max_mib << 20):
            back.zero_()

            def se():
                ctx.unpack_batch_into(packed, poffs, offs, back, st)

            t_se = timed(se, max(1, a.reps // 2))
            rec.update({"serial_ms": round(t_se * 1e3, 3),
                        "serial_GiBps": round(ub / t_se / 2**30, 1),
                        "serial_ok": bool(torch.equal(back, words))})
        if a.corrupt and n > 1:
            bad = torch.arange(n + 1, device="cuda") > n // 2
            offs2 = offs + bad.to(offs.dtype)  # chunk n/2 claims one word more
            back2 = torch.zeros(words.numel() + 1, dtype=torch.int64, device="cuda")

            def rs2():
                info["r2"] = ctx.unpack_batch_resync_into(packed, poffs, offs2, back2, st)

            t_rs2 = timed(rs2, a.reps)
            nbad = int((st != 0).sum().item())
            rec.update({"corrupt_resync_ms": round(t_rs2 * 1e3, 3), "corrupt_failed": nbad,
                        "corrupt_serial": info["r2"][1]})
            del back2, offs2
        print(json.dumps(rec), flush=True)
        del words, packed, back
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
