#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B=capnproto-rust_amd/build/abl
export CAPNP_UNPACK_KERNEL=tile
for pz in 1288490189 3435973837; do
timeout -k 10 200 python -u scripts/uvar.py capnproto-rust_amd/capnp_amd/libcapnp_packed.so $B/libcapnp_packed_u_p1.so $B/libcapnp_packed_u_p3.so --pz $pz --iters 5 &&
timeout -k 10 200 python -u scripts/uvar.py $B/libcapnp_packed_u_p3t4k.so --utc 32 --pz $pz --iters 5 || exit 1
done
