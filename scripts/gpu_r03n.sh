#!/bin/bash
# Pack variants: GPU tests on the default build, bench of each library, pack phase timeline.
#   scripts/gpu_r03n.sh <tag> <variant names under build/abl/libcapnp_packed_*.so>...
set -o pipefail
T=${1:-r03n}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L=capnproto-rust_amd/build/abl/libcapnp_packed_$v.so; fi
  CAPNP_PACKED_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench_$v.json 2>> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python scripts/bench_summary.py $v gpurun_out/${T}_bench_$v.json
done
timeout -k 10 120 python -u scripts/cs_prof.py --sync > gpurun_out/${T}_csprof.txt 2>&1 || { tail -20 gpurun_out/${T}_csprof.txt; exit 1; }
tail -4 gpurun_out/${T}_csprof.txt
