#!/bin/bash
# Round-2 traffic profiles: per-kernel read/write HBM bytes + kernel stats.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r02b}
bash scripts/traffic.sh gpurun_out/${T}_config2_sync --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_config2_sync.txt 2>&1 || { cat gpurun_out/${T}_config2_sync.txt; exit 1; }
bash scripts/traffic.sh gpurun_out/${T}_config2_nosync --steps 3 --warmup 1 --no-cpu --no-sync > gpurun_out/${T}_config2_nosync.txt 2>&1 || exit 1
bash scripts/traffic.sh gpurun_out/${T}_config3_sync --steps 3 --warmup 1 --no-cpu --workload config3 > gpurun_out/${T}_config3_sync.txt 2>&1 || exit 1
bash scripts/traffic.sh gpurun_out/${T}_carsales_sync --steps 3 --warmup 1 --no-cpu --workload carsales > gpurun_out/${T}_carsales_sync.txt 2>&1 || exit 1
cat gpurun_out/${T}_*.txt
