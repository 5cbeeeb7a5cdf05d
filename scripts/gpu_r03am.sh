#!/bin/bash
# Index-free unpack descriptors from the spec walk's record-start mask
# (UNPACK_DESC_MASK): full suite on the variant, interleaved A/B.
set -o pipefail
T=${1:-r03am}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_u_dmask.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_dm.log 2>&1 \
  || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests_dm.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests_dm.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_u_dmask.so"
for w in config2 carsales config3; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
