#!/bin/bash
# LDS / wave counters of one library build's kernels on a bench workload
# (diagnostic; one rocprofv3 --pmc pass per library, run on the GPU box):
#   scripts/lib_pmc.sh OUTDIR WORKLOAD LIB.so [LIB.so ...]
set -euo pipefail
OUT=$1; WL=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU \
    -d "$OUT/$n" -o run --output-format csv -- python3 scripts/wt_ablate.py --wl=$WL "$lib" > "$OUT/$n.log" 2>&1
  echo "== $n"
  python3 scripts/pmc_table.py "$OUT/$n" unpack_fit pack_cs pack_wt unpack_wt k_tile | tee "$OUT/$n.txt"
done
