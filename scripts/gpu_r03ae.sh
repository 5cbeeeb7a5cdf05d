#!/bin/bash
# Product library suite again (r03ad's variant run timed out in
# test_batch_long_runs), then the early-group A/B and resync round counts.
set -o pipefail
T=${1:-r03ae}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_earlyg.so"
for w in config2 carsales; do
  WL=$w timeout -k 10 300 python -u scripts/wt_ablate.py $L $L > gpurun_out/${T}_ab_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/${T}_ab_$w.log
done
for v in prof3 p_prof3eg; do
  timeout -k 10 120 python -u scripts/cs_prof.py --sync --lib $A/libcapnp_packed_$v.so > gpurun_out/${T}_$v.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${T}_$v.txt | grep -A3 "iter 2"
done
timeout -k 10 300 python -u scripts/resync_prof.py --lib $A/libcapnp_packed_f_rprof.so > gpurun_out/${T}_rprof.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_rprof.txt; exit 1; }
echo "== rprof"; grep -v amdgpu.ids gpurun_out/${T}_rprof.txt
