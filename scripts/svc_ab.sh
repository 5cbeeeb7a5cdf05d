#!/bin/bash
# A/B of the per-call service variants on one box, interleaved: the one-launch
# path (CAPNP_PERCALL_SERVICE=0), the product library and the variants under
# capnproto-rust_amd/build/abl/ named on the command line.
#   [SIZES=128,1500] bash scripts/svc_ab.sh OUT p1 p2 ...
out=$1; shift
sizes=${SIZES:-128,1500}
: > "$out"
for round in 1 2; do
  echo "{\"variant\": \"oneshot\", \"round\": $round}" >> "$out"
  CAPNP_PERCALL_SERVICE=0 timeout -k 10 120 python3 -u scripts/percall_bench.py --sizes $sizes 2>/dev/null >> "$out" || exit 1
  echo "{\"variant\": \"product\", \"round\": $round}" >> "$out"
  timeout -k 10 120 python3 -u scripts/percall_bench.py --sizes $sizes 2>/dev/null >> "$out" || exit 1
  for v in "$@"; do
    echo "{\"variant\": \"$v\", \"round\": $round}" >> "$out"
    timeout -k 10 120 python3 -u scripts/percall_bench.py --sizes $sizes \
      --lib capnproto-rust_amd/build/abl/libcapnp_packed_$v.so 2>/dev/null >> "$out" || exit 1
  done
done
