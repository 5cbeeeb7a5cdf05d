#!/bin/bash
# Parity tests (optional) then interleaved A/B of build/abl variants vs the product library
# (workload[:chunk_words], e.g. config2:100).
#   scripts/gpu_ab.sh <tag> <pytest targets or "-"> [workloads...]
set -o pipefail
TAG=${1:-ab}; T=${2:--}; shift 2 || true
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(config2)
mkdir -p gpurun_out
if [ "$T" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
for w in "${WL[@]}"; do
  echo "== $w"
  WL=${w%%:*} CW=$( [[ $w == *:* ]] && echo ${w##*:} || echo 128 ) timeout -k 10 300 python -u scripts/wt_ablate.py > gpurun_out/${TAG}_ab_$w.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_$w.log; exit 1; }
  cat gpurun_out/${TAG}_ab_$w.log
done
