#!/bin/bash
# Round-end check of the committed tree as the driver runs it: GPU suite,
# smoke(), the default bench line.
set -o pipefail
T=${1:-r03end}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py default gpurun_out/${T}_bench.json
