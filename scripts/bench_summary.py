#!/usr/bin/env python3
"""One line of the bench JSON's kernel times: bench_summary.py LABEL FILE."""
import json
import sys

d = json.load(open(sys.argv[2]))
k = d["kernels"]
print(sys.argv[1], d["value"], "pack", k["pack"]["ms"],
      "pack_ns", k.get("pack_nosync", {}).get("ms"), "unpack", k["unpack"]["ms"],
      "nosync", k.get("unpack_nosync", {}).get("ms"), "rt_noindex",
      d.get("roundtrip_noindex_GiBps"), "ok", d["roundtrip_ok"])
