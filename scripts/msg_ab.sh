# A/B of library variants on the message batch framing (scripts/msg_bench.py)
# and an index-free batch of 64-word chunks; variants from `make variant`
set -o pipefail
for rep in 1 2; do
for v in product "$@"; do
  if [ $v = product ]; then LIBP=capnproto-rust_amd/capnp_amd/libcapnp_packed.so; else LIBP=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
  echo "== $v" >> gpurun_out/msg_ab.txt
  CAPNP_PACKED_LIB=$LIBP timeout -k 10 100 python -u scripts/msg_bench.py 2>/dev/null | grep -v amdgpu >> gpurun_out/msg_ab.txt || exit 1
  CAPNP_PACKED_LIB=$LIBP CW=64 timeout -k 10 100 python -u scripts/wt_ablate.py --wl=config2 $LIBP 2>/dev/null | grep nosync >> gpurun_out/msg_ab.txt || exit 1
done
done
