#!/bin/bash
# Kernel trace + PMC passes of the default bench workload (run on the GPU box).
#   scripts/profile.sh <outdir> [bench args...]
# Each rocprofv3 pass is its own run (counters never combined with tracing).
set -euo pipefail
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 5 --warmup 1 --no-cpu)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d "$OUT/sq1" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d "$OUT/sq2" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d "$OUT/sq3" -o run --output-format csv \
  -- python3 bench.py "${ARGS[@]}" > "$OUT/sq3.log" 2>&1
python3 scripts/summarize_prof.py "$OUT" pack_cs_kernel pack_ovf_kernel unpack_fit_kernel unpack_ovf_kernel unpack_ovf_win_kernel > "$OUT/summary.txt"
cat "$OUT/summary.txt"
echo "profile done: $OUT"
