#!/bin/bash
# Product suite after reverting the resync k_tile restructure (r03ad/r03ae
# timed out in resync-path tests), then the default bench line.
set -o pipefail
T=${1:-r03af}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py default gpurun_out/${T}_bench.json
