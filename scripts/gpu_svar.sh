#!/bin/bash
# stream-unpack variant timing (scripts/uvar.py over build/abl/libcapnp_packed_s_*.so)
set -o pipefail
mkdir -p gpurun_out
L=$(ls capnproto-rust_amd/build/abl/libcapnp_packed_s_*.so)
timeout -k 10 300 python -u scripts/uvar.py $L --iters 5 > gpurun_out/${1:-sv}_pz30.txt 2>&1 && cat gpurun_out/${1:-sv}_pz30.txt &&
timeout -k 10 300 python -u scripts/uvar.py $L --iters 5 --pz 3435973837 > gpurun_out/${1:-sv}_pz80.txt 2>&1 && cat gpurun_out/${1:-sv}_pz80.txt
