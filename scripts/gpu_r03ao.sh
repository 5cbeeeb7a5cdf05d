#!/bin/bash
# Look-back knobs re-checked with the early group aggregate: group of 32
# tiles (PACK_GROUP), group-record window 32 / 8 (PACK_GWIN); pack parity of
# the group-32 build, interleaved A/B.
set -o pipefail
T=${1:-r03ao}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_g32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pack_many_tiles.py tests/test_gpu_wordtiles.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests_g32.log 2>&1 || { tail -30 gpurun_out/${T}_tests_g32.log; exit 1; }
tail -1 gpurun_out/${T}_tests_g32.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_g32.so $A/libcapnp_packed_p_gwin32.so $A/libcapnp_packed_p_gwin8.so"
for w in config2 carsales; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
