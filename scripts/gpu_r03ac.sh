#!/bin/bash
# Resync block->chunk map (RESYNC_BLKC) and segment units: GPU suite on the
# combined variant, config-4 A/B, resync and pack phase timelines.
set -o pipefail
T=${1:-r03ac}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_f_blkc.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_blkc.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests_blkc.log; exit 1; }
tail -1 gpurun_out/${T}_tests_blkc.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_f_blkc.so"
WL=config4 timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_config4.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ab_config4.log; exit 1; }
echo "== config4"; grep -v amdgpu.ids gpurun_out/${T}_ab_config4.log
timeout -k 10 300 python -u scripts/resync_prof.py --lib $A/libcapnp_packed_f_rprof.so > gpurun_out/${T}_rprof.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_rprof.txt; exit 1; }
echo "== rprof"; grep -v amdgpu.ids gpurun_out/${T}_rprof.txt
timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/libcapnp_packed_prof3.so > gpurun_out/${T}_prof3.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_prof3.txt; exit 1; }
echo "== prof3"; grep -v amdgpu.ids gpurun_out/${T}_prof3.txt
