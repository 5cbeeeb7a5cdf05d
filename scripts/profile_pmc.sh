#!/bin/bash
# One rocprofv3 --pmc pass per counter group over the bench workload.
#   [BENCH_ARGS="--workload config4"] scripts/profile_pmc.sh <outdir> "<group1 counters>" ...
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/g$i" -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$OUT/g$i.log" 2>&1
done
python3 scripts/summarize_prof.py "$OUT"
