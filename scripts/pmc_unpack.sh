#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over scripts/uvar.py.
#   scripts/pmc_unpack.sh <outdir> <uvar args...>
set -uo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_ADDR_CONFLICT"
G3="SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
i=0
for grp in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/g$i" -o run --output-format csv \
    -- python3 scripts/uvar.py --iters 2 "$@" > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/g$i.log"; exit 1; }
done
python3 scripts/summarize_prof.py "$OUT" unpack_sync_kernel unpack_kernel
