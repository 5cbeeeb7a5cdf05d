#!/bin/bash
# Index-free unpack variants: GPU tests on the default build, bench of both.
set -o pipefail
T=${1:-r03h}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for v in default merged pair both; do
  if [ $v = default ]; then L=""; else L=capnproto-rust_amd/build/abl/libcapnp_packed_u_$v.so; fi
  CAPNP_PACKED_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench_$v.json 2>> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python scripts/bench_summary.py $v gpurun_out/${T}_bench_$v.json
done
timeout -k 10 180 python -u scripts/unpack_prof.py > gpurun_out/${T}_uprof.txt 2>&1 || { tail -20 gpurun_out/${T}_uprof.txt; exit 1; }
tail -1 gpurun_out/${T}_uprof.txt
