#!/bin/bash
# Plan kernel back at the 64-word window (branch-free loads) with the word-tile
# kernel's batched scalar loads: product suite, config-4 A/B against the 16-word window.
set -o pipefail
T=${1:-r03ai}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { grep -E "PASSED|FAILED|Timeout" gpurun_out/${T}_tests.log | tail -5; exit 1; }
tail -1 gpurun_out/${T}_tests.log
CAPNP_PACKED_LIB=$A/libcapnp_packed_p_win16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wordtiles.py \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests_win16.log 2>&1 \
  || { tail -20 gpurun_out/${T}_tests_win16.log; exit 1; }
tail -1 gpurun_out/${T}_tests_win16.log
L="capnproto-rust_amd/capnp_amd/libcapnp_packed.so $A/libcapnp_packed_p_win16.so"
WL=config4 timeout -k 10 300 python -u scripts/wt_ablate.py $L > gpurun_out/${T}_ab_config4.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ab_config4.log; exit 1; }
echo "== config4"; grep -v amdgpu.ids gpurun_out/${T}_ab_config4.log
bash scripts/traffic.sh gpurun_out/${T}_config4_sync --steps 3 --warmup 1 --no-cpu --workload config4 > gpurun_out/${T}_config4_sync.txt 2>&1 \
  || { cat gpurun_out/${T}_config4_sync.txt; exit 1; }
grep -A4 "pack_wt_plan\|pack_wt_kernel<true>" gpurun_out/${T}_config4_sync.txt | head -20
timeout -k 10 300 python -u bench.py --workload config4 --no-cpu > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err \
  || { tail -20 gpurun_out/${T}_c4.err; exit 1; }
python scripts/bench_summary.py config4 gpurun_out/${T}_c4.json
