#!/bin/bash
# Round-end measurement set: GPU tests, bench lines per workload, then
# per-kernel traffic and kernel stats (scripts/traffic.sh).  scripts/gpu_final.sh <tag>
set -o pipefail
T=${1:-r02g}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for w in config2 config3 carsales config4; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err \
    || { tail -20 gpurun_out/${T}_${w}_bench.err; exit 1; }
  cat gpurun_out/${T}_${w}_bench.json
done
bash scripts/gpu_traffic_r02.sh $T > /dev/null || exit 1
bash scripts/traffic.sh gpurun_out/${T}_config4_sync --steps 3 --warmup 1 --no-cpu --workload config4 \
  > gpurun_out/${T}_config4_sync.txt 2>&1 || { cat gpurun_out/${T}_config4_sync.txt; exit 1; }
echo traffic done
