#!/bin/bash
# Round-2 GPU run: selected parity tests, then bench lines per workload.
#   scripts/gpu_r02.sh <tag> <pytest file/-k spec or "-"> [workloads...]
set -o pipefail
TAG=${1:-r02}; T=${2:--}; shift 2 || true
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(config2)
mkdir -p gpurun_out
if [ "$T" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -5 gpurun_out/${TAG}_tests.log
fi
for w in "${WL[@]}"; do
  extra=""; [ "$w" = "config5" ] && extra="--steps 10"
  timeout -k 10 400 python -u bench.py --workload $w $extra ${BENCH_ARGS:-} \
    > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail -20 gpurun_out/${TAG}_bench_$w.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$w.json
done
