set -o pipefail
# round-5 closing measurements: tests, every workload line, traffic and PMC of
# config 4 (its kernels changed since r05l), the long-unit phases
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/config2.json 2>$O/config2.err && python scripts/bench_summary.py c2 $O/config2.json &&
for w in config3 carsales config4; do timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/$w.json 2>/dev/null && python scripts/bench_summary.py $w $O/$w.json || exit 1; done &&
timeout -k 10 300 python bench.py --workload config3 --chunks 23400000 --steps 5 --warmup 1 --no-cpu > $O/config3_full.json 2>/dev/null && python scripts/bench_summary.py c3full $O/config3_full.json &&
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $O/config5.json 2>/dev/null && python scripts/bench_summary.py c5 $O/config5.json &&
bash scripts/traffic.sh $O/tr_c4 --workload config4 --steps 3 --warmup 1 --no-cpu > $O/tr_c4.txt 2>&1 &&
bash scripts/traffic.sh $O/tr_c2 > $O/tr_c2.txt 2>&1 &&
BENCH_ARGS="--workload config4" bash scripts/profile_pmc.sh $O/pmc_c4 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" > $O/pmc_c4.txt 2>&1 &&
timeout -k 10 300 python -u scripts/stream_bench.py > $O/stream.json 2>/dev/null &&
timeout -k 10 300 python -u scripts/resync_bench.py > $O/resync.txt 2>&1 &&
timeout -k 10 400 python -u scripts/dropin_bench.py > $O/dropin.txt 2>&1 && echo done
