#!/bin/bash
# Copy-out with the LDS reads first (PACK_COPY_PRE): pack parity on the
# variant, interleaved A/B, timelines.
set -o pipefail
T=${1:-r03al}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_copypre.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pack_many_tiles.py tests/test_gpu_carsales.py tests/test_gpu_messages.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_cp.log 2>&1 \
  || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests_cp.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests_cp.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_copypre.so"
for w in config2 carsales config3; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
for v in prof3 p_prof3cp; do
  timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/libcapnp_packed_$v.so > gpurun_out/${T}_$v.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${T}_$v.txt | grep -A3 "iter 2"
done
