#!/bin/bash
# Bench one workload and a rocprofv3 kernel-stats pass of the same command:
#   scripts/gpu_prof.sh <tag> <workload> [bench args...]
set -o pipefail
TAG=$1; W=$2; shift 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python -u bench.py --workload $W --no-cpu "$@" \
  > gpurun_out/${TAG}_bench_$W.json 2> gpurun_out/${TAG}_bench_$W.err || { tail -20 gpurun_out/${TAG}_bench_$W.err; exit 1; }
cat gpurun_out/${TAG}_bench_$W.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$W -o run -- \
  python -u bench.py --workload $W --no-cpu --steps 5 --warmup 2 "$@" \
  > gpurun_out/${TAG}_prof_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof_$W.log; exit 1; }
f=$(find gpurun_out/${TAG}_prof_$W -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -15
