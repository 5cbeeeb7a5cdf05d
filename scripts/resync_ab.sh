#!/bin/bash
# Interleaved A/B of the index-free decode (scripts/resync_bench.py) between
# the product library and variants under capnproto-rust_amd/build/abl/:
#   [WL=config4_1GiB,...] bash scripts/resync_ab.sh OUT variant...
out=$1; shift
wl=${WL:-config4_1GiB,config4k0_1GiB,config4k2_1GiB}
: > "$out"
for round in 1 2; do
  for v in product "$@"; do
    if [ "$v" = product ]; then lib=""; else lib=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
    echo "{\"variant\": \"$v\", \"round\": $round}" >> "$out"
    CAPNP_PACKED_LIB=$lib timeout -k 10 300 python3 -u scripts/resync_bench.py --workloads "$wl" --serial-max-mib 0 >> "$out" 2>/dev/null || exit 1
  done
done
