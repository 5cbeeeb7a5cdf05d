#!/bin/bash
# Index-free segment walk lead-in re-checked on the final tree
# (UNPACK_SEG_OVERLAP 40 / 56 / 64 vs 48): parity of the variants' index-free
# paths, interleaved A/B.
set -o pipefail
T=${1:-r03at}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
for v in ov40 ov56 ov64; do
  CAPNP_PACKED_LIB=$A/libcapnp_packed_u_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_garbage.py tests/test_gpu_messages.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_tests_$v.log 2>&1 || { tail -30 gpurun_out/${T}_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${T}_tests_$v.log)"
done
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_u_ov40.so $A/libcapnp_packed_u_ov56.so $A/libcapnp_packed_u_ov64.so"
for w in config2 carsales; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
