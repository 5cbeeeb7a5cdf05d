#!/bin/bash
# Resync lead-in 64 / 80 / 96 vs 48 (RESYNC_LEAD): resync / discovery parity on
# the variants, config-4 A/B.
set -o pipefail
T=${1:-r03as}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
for v in lead64 lead80 lead96; do
  CAPNP_PACKED_LIB=$A/libcapnp_packed_f_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_resync.py \
    tests/test_gpu_find_messages.py tests/test_gpu_async.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_tests_$v.log 2>&1 || { tail -30 gpurun_out/${T}_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${T}_tests_$v.log)"
done
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_f_lead64.so $A/libcapnp_packed_f_lead80.so $A/libcapnp_packed_f_lead96.so"
WL=config4 timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_config4.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ab_config4.log; exit 1; }
echo "== config4"; grep -v amdgpu.ids gpurun_out/${T}_ab_config4.log
