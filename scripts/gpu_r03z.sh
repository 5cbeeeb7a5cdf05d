#!/bin/bash
# New defaults (one-round-trip prologues) + segment-unit resync variant:
# GPU suites on both, config-4 A/B, default bench line.
set -o pipefail
T=${1:-r03z}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
CAPNP_PACKED_LIB=$A/libcapnp_packed_f_all.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_all.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests_all.log; exit 1; }
tail -1 gpurun_out/${T}_tests_all.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_f_all.so"
WL=config4 timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_config4.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ab_config4.log; exit 1; }
echo "== config4"; grep -v amdgpu.ids gpurun_out/${T}_ab_config4.log
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py default gpurun_out/${T}_bench.json
