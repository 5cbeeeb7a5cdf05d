#!/bin/bash
# Round-3 final measurement set, part B: per-call HBM traffic (FETCH / WRITE
# passes) for every workload, and the pack PMC counters of config 2.
set -o pipefail
T=${1:-r03fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/traffic.sh gpurun_out/${T}_config2_sync --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_config2_sync.txt 2>&1 || { cat gpurun_out/${T}_config2_sync.txt; exit 1; }
bash scripts/traffic.sh gpurun_out/${T}_config2_nosync --steps 3 --warmup 1 --no-cpu --no-sync > gpurun_out/${T}_config2_nosync.txt 2>&1 || { cat gpurun_out/${T}_config2_nosync.txt; exit 1; }
bash scripts/traffic.sh gpurun_out/${T}_config3_sync --steps 3 --warmup 1 --no-cpu --workload config3 > gpurun_out/${T}_config3_sync.txt 2>&1 || { cat gpurun_out/${T}_config3_sync.txt; exit 1; }
bash scripts/traffic.sh gpurun_out/${T}_carsales_sync --steps 3 --warmup 1 --no-cpu --workload carsales > gpurun_out/${T}_carsales_sync.txt 2>&1 || { cat gpurun_out/${T}_carsales_sync.txt; exit 1; }
bash scripts/traffic.sh gpurun_out/${T}_config4_sync --steps 3 --warmup 1 --no-cpu --workload config4 > gpurun_out/${T}_config4_sync.txt 2>&1 || { cat gpurun_out/${T}_config4_sync.txt; exit 1; }
cat gpurun_out/${T}_*_sync.txt gpurun_out/${T}_config2_nosync.txt
bash scripts/profile_pmc.sh gpurun_out/${T}_pmc "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" > gpurun_out/${T}_pmc.txt 2>&1 || { tail -30 gpurun_out/${T}_pmc.txt; exit 1; }
cat gpurun_out/${T}_pmc.txt
