#!/bin/bash
# Round-3 baseline: GPU tests, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03a_tests.log 2>&1 || { tail -30 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 \
  || { tail -20 gpurun_out/r03a_smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err \
  || { tail -20 gpurun_out/r03a_bench.err; exit 1; }
cat gpurun_out/r03a_bench.json
