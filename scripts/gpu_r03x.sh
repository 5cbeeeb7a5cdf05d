#!/bin/bash
# Multi-level look-back (PACK_LB=2): parity of the variant, interleaved A/B, phase timelines.
set -o pipefail
T=${1:-r03x}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_lb2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pack_many_tiles.py tests/test_gpu_carsales.py tests/test_gpu_wordtiles.py tests/test_gpu_messages.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_lb2.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests_lb2.log; exit 1; }
tail -1 gpurun_out/${T}_tests_lb2.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_lb2.so $A/libcapnp_packed_p_lb2s1.so"
for w in config2 carsales config3 config4; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; cat gpurun_out/${T}_ab_$w.log
done
for v in lb1 lb2; do
  timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/prof3_$v.so > gpurun_out/${T}_prof_$v.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_prof_$v.txt; exit 1; }
  echo "== prof $v"; grep -v amdgpu.ids gpurun_out/${T}_prof_$v.txt
done
