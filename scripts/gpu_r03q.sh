#!/bin/bash
# One-pass stream decode: GPU tests, the 1 GiB carsales stream bench, config 2 / 4 bench lines.
set -o pipefail
T=${1:-r03q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_find_messages.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_find.log 2>&1 || { tail -40 gpurun_out/${T}_find.log; exit 1; }
tail -3 gpurun_out/${T}_find.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u scripts/stream_bench.py > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err \
  || { tail -20 gpurun_out/${T}_stream.err; exit 1; }
cat gpurun_out/${T}_stream.json
for w in config2 config4; do
  timeout -k 10 300 python -u bench.py --no-cpu --workload $w > gpurun_out/${T}_bench_$w.json 2>> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python scripts/bench_summary.py $w gpurun_out/${T}_bench_$w.json
done
