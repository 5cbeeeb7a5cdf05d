#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B=capnproto-rust_amd/build/abl
for pz in 1288490189 3435973837; do
timeout -k 10 200 python -u scripts/uvar.py capnproto-rust_amd/capnp_amd/libcapnp_packed.so $B/libcapnp_packed_u_w6.so $B/libcapnp_packed_u_w7.so --sync --pz $pz --iters 8 || exit 1
done
