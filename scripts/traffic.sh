#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) and a kernel trace over
# the bench workload, summarised per kernel (read / write split).
#   scripts/traffic.sh <outdir> [bench args...]
set -uo pipefail
OUT=$1; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 3 --warmup 1 --no-cpu)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/write.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/trace.log" 2>&1 || exit 1
python3 scripts/summarize_prof.py "$OUT" pack_cs_kernel pack_kernel pack_ovf_kernel unpack_fit_kernel unpack_ovf_kernel unpack_ovf_win_kernel unpack_kernel k_tile k_cut \
  pack_wt_kernel pack_wt_plan unpack_wt_kernel unpack_wt_plan unpack_wt_finish --json "$OUT/traffic.json"
