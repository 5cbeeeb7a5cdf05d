#!/bin/bash
# Resync tile resolution: phase profile, segments-per-block A/B on config 4.
set -o pipefail
T=${1:-r03aa}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 300 python -u scripts/resync_prof.py --lib $A/libcapnp_packed_f_rprof.so > gpurun_out/${T}_rprof.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_rprof.txt; exit 1; }
cat gpurun_out/${T}_rprof.txt
for v in segs2 segs8; do
  CAPNP_PACKED_LIB=$A/libcapnp_packed_f_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_resync.py tests/test_gpu_find_messages.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/${T}_tests_$v.log; exit 1; }
  tail -1 gpurun_out/${T}_tests_$v.log
done
for v in default segs2 segs8; do
  if [ $v = default ]; then L=""; else L=$A/libcapnp_packed_f_$v.so; fi
  CAPNP_PACKED_LIB=$L timeout -k 10 300 python -u bench.py --workload config4 --no-cpu --steps 5 --warmup 1 > gpurun_out/${T}_c4_$v.json 2>> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python scripts/bench_summary.py $v gpurun_out/${T}_c4_$v.json
done
