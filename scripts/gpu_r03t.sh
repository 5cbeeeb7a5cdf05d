#!/bin/bash
# Round-3 artifacts: adaptor throughput, kernel trace + PMC summary of the default bench.
set -o pipefail
T=${1:-r03t}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/adaptor_bench.py > gpurun_out/${T}_adaptor.json 2> gpurun_out/${T}_adaptor.err \
  || { tail -20 gpurun_out/${T}_adaptor.err; exit 1; }
cat gpurun_out/${T}_adaptor.json
timeout -k 10 900 bash scripts/profile.sh gpurun_out/${T}_prof > gpurun_out/${T}_prof.log 2>&1 || { tail -30 gpurun_out/${T}_prof.log; exit 1; }
tail -60 gpurun_out/${T}_prof.log
