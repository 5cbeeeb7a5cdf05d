#!/bin/bash
# Round-2 final profiles: per workload a bench line (with the CPU baseline),
# a rocprofv3 kernel-stats pass and the FETCH/WRITE traffic passes.
#   scripts/gpu_r02c.sh <tag> [workloads...]
set -o pipefail
T=${1:-r02c}; shift
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(config2 config3 carsales config4)
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in "${WL[@]}"; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/${T}_bench_$w.json 2> gpurun_out/${T}_bench_$w.err \
    || { tail -20 gpurun_out/${T}_bench_$w.err; exit 1; }
  cat gpurun_out/${T}_bench_$w.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_$w -o run -- \
    python3 -u bench.py --workload $w --no-cpu --steps 5 --warmup 2 > gpurun_out/${T}_prof_$w.log 2>&1 \
    || { tail -20 gpurun_out/${T}_prof_$w.log; exit 1; }
  bash scripts/traffic.sh gpurun_out/${T}_traffic_$w --steps 3 --warmup 1 --no-cpu --workload $w \
    > gpurun_out/${T}_traffic_$w.txt 2>&1 || { tail -20 gpurun_out/${T}_traffic_$w.txt; exit 1; }
done
bash scripts/traffic.sh gpurun_out/${T}_traffic_config2_nosync --steps 3 --warmup 1 --no-cpu --no-sync \
  > gpurun_out/${T}_traffic_config2_nosync.txt 2>&1 || exit 1
echo done
