#!/bin/bash
# Round-3 batch: GPU tests, bench, stream-adaptor throughput (1 MiB calls).
set -o pipefail
T=${1:-r03v}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u scripts/adaptor_bench.py > gpurun_out/${T}_adaptor.json 2> gpurun_out/${T}_adaptor.err \
  || { tail -20 gpurun_out/${T}_adaptor.err; exit 1; }
cat gpurun_out/${T}_adaptor.json
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py default gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4 -o run --output-format csv \
  -- python3 bench.py --workload config4 --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err \
  || { tail -20 gpurun_out/${T}_c4.err; exit 1; }
python scripts/bench_summary.py config4 gpurun_out/${T}_c4.json
