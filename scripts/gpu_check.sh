#!/bin/bash
# GPU-box check: parity tests, then a short bench line (no CPU leg).
# usage: scripts/gpu_check.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${K:+-k "$K"} > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
cat gpurun_out/b.log
