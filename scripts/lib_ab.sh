#!/bin/bash
# Interleaved bench.py A/B of the product library against variants under
# capnproto-rust_amd/build/abl/ (CAPNP_PACKED_LIB), two rounds:
#   bash scripts/lib_ab.sh OUT WORKLOAD variant...
out=$1; wl=$2; shift 2
: > "$out"
for round in 1 2; do
  for v in product "$@"; do
    if [ "$v" = product ]; then lib=""; else lib=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
    echo "{\"variant\": \"$v\", \"round\": $round}" >> "$out"
    CAPNP_PACKED_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload "$wl" --steps 20 --warmup 3 --no-cpu >> "$out" 2>/dev/null || exit 1
  done
done
