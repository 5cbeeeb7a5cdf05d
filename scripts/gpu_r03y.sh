#!/bin/bash
# One-round-trip prologues (PACK_CS_SPEC, UNPACK_PRO): full GPU suite on the
# variant library, interleaved A/B against the product library, pack timeline.
set -o pipefail
T=${1:-r03y}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
CAPNP_PACKED_LIB=$A/libcapnp_packed_f_new.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_new.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests_new.log; exit 1; }
tail -1 gpurun_out/${T}_tests_new.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_spec.so $A/libcapnp_packed_u_pro.so $A/libcapnp_packed_f_new.so"
for w in config2 carsales config3; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/prof3_spec.so > gpurun_out/${T}_prof_spec.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_prof_spec.txt; exit 1; }
echo "== prof spec"; grep -v amdgpu.ids gpurun_out/${T}_prof_spec.txt
