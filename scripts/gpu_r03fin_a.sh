#!/bin/bash
# Round-3 final measurement set, part A: GPU suite, one bench line per
# workload (CPU baselines in the same run), kernel stats of the default line.
set -o pipefail
T=${1:-r03fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for w in config2 config3 carsales config4; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err \
    || { tail -20 gpurun_out/${T}_${w}_bench.err; exit 1; }
  python scripts/bench_summary.py $w gpurun_out/${T}_${w}_bench.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c2 -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_c2_prof.json 2> gpurun_out/${T}_c2_prof.err \
  || { tail -20 gpurun_out/${T}_c2_prof.err; exit 1; }
python scripts/bench_summary.py prof gpurun_out/${T}_c2_prof.json
timeout -k 10 300 python -u scripts/stream_bench.py > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err \
  || { tail -20 gpurun_out/${T}_stream.err; exit 1; }
cat gpurun_out/${T}_stream.json
