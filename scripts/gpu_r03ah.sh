#!/bin/bash
# PACK_EARLYG=1 as the product; EARLYG=2 (inclusive record published early
# too) and EARLYG=0 as variants: parity, interleaved A/B, timelines.
set -o pipefail
T=${1:-r03ah}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests.log
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_eg2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pack_many_tiles.py tests/test_gpu_carsales.py tests/test_gpu_messages.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_eg2.log 2>&1 \
  || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests_eg2.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests_eg2.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_eg2.so $A/libcapnp_packed_p_eg0.so"
for w in config2 carsales config3; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
for v in prof3 p_prof3eg2; do
  timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/libcapnp_packed_$v.so > gpurun_out/${T}_$v.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${T}_$v.txt | grep -A3 "iter 2"
done
