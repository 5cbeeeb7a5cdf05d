#!/bin/bash
# GPU test run: scripts/gpu_tests.sh <tag> [pytest targets...]
set -o pipefail
TAG=${1:-t}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -40 gpurun_out/${TAG}_tests.log
exit $rc
