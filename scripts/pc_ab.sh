set -o pipefail
for rep in 1 2; do
for v in product direct split64 both; do
  if [ $v = product ]; then LIBP=capnproto-rust_amd/capnp_amd/libcapnp_packed.so; else LIBP=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
  echo "== $v" >> gpurun_out/r05z_pc_ab.txt
  CAPNP_PACKED_LIB=$LIBP timeout -k 10 60 python -u scripts/percall_bench.py --sizes 128,256,512,1500 --reps 300 2>/dev/null | grep words >> gpurun_out/r05z_pc_ab.txt || exit 1
done
done
