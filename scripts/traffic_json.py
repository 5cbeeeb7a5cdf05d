#!/usr/bin/env python3
"""Per-call HBM traffic of the bench's three API calls, from scripts/traffic.sh
output dirs, merged into profiles/traffic.json (read by bench.py for the
roofline's `traffic`).

    traffic_json.py profiles/traffic.json KEY=DIR [KEY=DIR ...]

KEY is bench.py's lookup key, "<workload>:<chunks>x<words>[:sync]".  A call
may launch several kernels (word tiles: bits/map/plan/kernel/fix_sync; the
split sync unpack: fit + overflow; index-free long chunks: the resync
kernels); its traffic is the sum of their per-launch means.  read = 2 x
FETCH_SIZE (gfx950 FETCH reports half, MI355X_MICROARCH.md), write =
WRITE_SIZE, KiB -> bytes.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

PACK = {"pack_kernel", "pack_cs_kernel", "pack_lean_kernel", "pack_ovf_kernel", "pack_wt_bits",
        "pack_wt_map", "pack_wt_plan", "pack_wt_kernel", "pack_wt_fix_sync"}
PACK_SYNC_TEMPLATED = {"pack_kernel", "pack_cs_kernel", "pack_lean_kernel", "pack_wt_kernel"}
UNPACK_SYNC = {"unpack_fit_kernel", "unpack_ovf_kernel", "unpack_wt_plan", "unpack_wt_kernel",
               "unpack_wt_finish", "unpack_kernel<true>"}


def _strip(name):
    return re.sub(r"^void\s+", "", name).replace("(anonymous namespace)::", "")


def templ(name):
    name = _strip(name)
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*(<[^()]*>)?)\s*\(", name)
    return m.group(1) if m else name


def role(t):
    bare = t.split("<")[0]
    if bare == "k_check_offsets":  # (the C ABI's offset validation, every call)
        return None
    if bare in PACK_SYNC_TEMPLATED and t.startswith(bare + "<false"):
        return "pack_nosync"  # (bench.py times the index-free pack too)
    if bare in PACK:
        return "pack"
    if bare in ("unpack_fit_kernel", "unpack_ovf_kernel", "unpack_ovf_win_kernel") and t.endswith("<false>"):
        return "unpack_nosync"
    if bare in UNPACK_SYNC or t in UNPACK_SYNC:
        return "unpack"
    if t == "unpack_kernel<false>" or bare.startswith("k_"):
        return "unpack_nosync"
    return None


def per_kernel(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[templ(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, dct in agg.items():
        if "FETCH_SIZE" in dct and "WRITE_SIZE" in dct:
            rd = 2 * 1024 * sum(dct["FETCH_SIZE"]) / len(dct["FETCH_SIZE"])
            wr = 1024 * sum(dct["WRITE_SIZE"]) / len(dct["WRITE_SIZE"])
            out[k] = (rd, wr)
    return out


def main():
    path = sys.argv[1]
    tj = json.load(open(path)) if os.path.exists(path) else {}
    for arg in sys.argv[2:]:
        key, d = arg.split("=", 1)
        ent = {}
        for k, (rd, wr) in sorted(per_kernel(d).items()):
            r = role(k)
            if r is None:
                continue
            e = ent.setdefault(r, {"read": 0, "write": 0, "total": 0, "kernels": {}})
            e["read"] += int(rd)
            e["write"] += int(wr)
            e["total"] += int(rd + wr)
            e["kernels"][k] = {"read": int(rd), "write": int(wr)}
        if not key.endswith(":sync"):  # the index-free run's only encode / decode
            if "unpack_nosync" in ent:
                ent["unpack"] = ent.pop("unpack_nosync")
            if "pack_nosync" in ent:
                ent["pack"] = ent.pop("pack_nosync")
        tj[key] = ent
        print(key, {r: (round(e["read"] / 1e6, 1), round(e["write"] / 1e6, 1))
                    for r, e in ent.items()})
    json.dump(tj, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
