#!/bin/bash
# Early group aggregate in the word-tile kernel (PACK_WT_EARLYG): word-tile
# parity on the variant, config-4 A/B.
set -o pipefail
T=${1:-r03ap}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_wteg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_wordtiles.py \
  tests/test_gpu_parity.py tests/test_gpu_pack_many_tiles.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests_wteg.log 2>&1 || { tail -30 gpurun_out/${T}_tests_wteg.log; exit 1; }
tail -1 gpurun_out/${T}_tests_wteg.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_wteg.so"
WL=config4 timeout -k 10 300 python -u scripts/wt_ablate.py $L $L > gpurun_out/${T}_ab_config4.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ab_config4.log; exit 1; }
echo "== config4"; grep -v amdgpu.ids gpurun_out/${T}_ab_config4.log
