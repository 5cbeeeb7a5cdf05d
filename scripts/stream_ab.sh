# A/B of library variants on the foreign-stream decode (scripts/stream_bench.py),
# two alternating passes; variants from `make variant`, named as arguments
set -o pipefail
for rep in 1 2; do
for v in product "$@"; do
  if [ $v = product ]; then LIBP=capnproto-rust_amd/capnp_amd/libcapnp_packed.so; else LIBP=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
  echo "== $v $(CAPNP_PACKED_LIB=$LIBP timeout -k 10 100 python -u scripts/stream_bench.py --reps 3 2>/dev/null | tail -1)" >> gpurun_out/stream_ab.txt || exit 1
done
done
