#!/bin/bash
# Tile-wide rounds: GPU tests, phase profile, config-4 bench, foreign stream bench, adaptor.
set -o pipefail
T=${1:-r03ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u scripts/resync_prof.py --lib $A/libcapnp_packed_f_rprof.so > gpurun_out/${T}_rprof.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_rprof.txt; exit 1; }
cat gpurun_out/${T}_rprof.txt
timeout -k 10 300 python -u bench.py --workload config4 --no-cpu --steps 5 --warmup 1 > gpurun_out/${T}_c4.json 2>> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py config4 gpurun_out/${T}_c4.json
timeout -k 10 300 python -u scripts/stream_bench.py > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err \
  || { tail -20 gpurun_out/${T}_stream.err; exit 1; }
cat gpurun_out/${T}_stream.json
