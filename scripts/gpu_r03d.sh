#!/bin/bash
# Tests, bench, cs pack phase timeline, PMC counters of the codec kernels.
set -o pipefail
T=${1:-r03d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); k=d['kernels']; print(d['value'], 'pack', k['pack']['ms'], 'unpack', k['unpack']['ms'], 'nosync', k['unpack_nosync']['ms'], d['roundtrip_ok'])"
timeout -k 10 120 python -u scripts/cs_prof.py --sync > gpurun_out/${T}_csprof.txt 2>&1 || { tail -20 gpurun_out/${T}_csprof.txt; exit 1; }
cat gpurun_out/${T}_csprof.txt
for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
            "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/$T/pmc$n -o run --output-format csv \
    -- python3 scripts/kernel_once.py --iters 3 > gpurun_out/$T/pmc$n.log 2>&1 || { tail -5 gpurun_out/$T/pmc$n.log; echo "pmc pass $n failed"; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/trace -o run --output-format csv \
  -- python3 scripts/kernel_once.py --iters 3 > gpurun_out/$T/trace.log 2>&1 || echo "trace failed"
python3 scripts/summarize_prof.py gpurun_out/$T pack_cs_kernel unpack_fit_kernel unpack_ovf_kernel > gpurun_out/$T/summary.txt 2>&1
cat gpurun_out/$T/summary.txt | head -60
