set -o pipefail
# round-6 closing measurements: tests, smoke, every workload line, traffic
# (FETCH/WRITE passes) for each workload, config-2 PMC, the drop-in,
# adaptor, long-unit, resync, stream and message benches
O=${OUTDIR:-gpurun_out/r06z}
mkdir -p $O
PART=${1:-1}
if [ "$PART" = 1 ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && tail -1 $O/smoke.txt &&
timeout -k 10 300 python bench.py > $O/config2.json 2>$O/config2.err && python scripts/bench_summary.py c2 $O/config2.json &&
for w in config3 carsales config4; do timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/$w.json 2>/dev/null && python scripts/bench_summary.py $w $O/$w.json || exit 1; done &&
timeout -k 10 300 python bench.py --workload config3 --chunks 23400000 --steps 5 --warmup 1 --no-cpu > $O/config3_full.json 2>/dev/null && python scripts/bench_summary.py c3full $O/config3_full.json &&
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $O/config5.json 2>/dev/null && python scripts/bench_summary.py c5 $O/config5.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $O/trace_c2.json 2> $O/trace_c2.err && python scripts/bench_summary.py prof $O/trace_c2.json && echo part1 done
elif [ "$PART" = 2 ]; then
bash scripts/traffic.sh $O/tr_c2 > $O/tr_c2.txt 2>&1 &&
bash scripts/traffic.sh $O/tr_c3 --workload config3 --steps 3 --warmup 1 --no-cpu > $O/tr_c3.txt 2>&1 &&
bash scripts/traffic.sh $O/tr_cs --workload carsales --steps 3 --warmup 1 --no-cpu > $O/tr_cs.txt 2>&1 &&
bash scripts/traffic.sh $O/tr_c4 --workload config4 --steps 3 --warmup 1 --no-cpu > $O/tr_c4.txt 2>&1 &&
timeout -k 10 1000 bash scripts/profile.sh $O/pmc_c2 > $O/pmc_c2.log 2>&1 && echo part2 done
else
timeout -k 10 300 python -u scripts/stream_bench.py > $O/stream.json 2>/dev/null &&
timeout -k 10 300 python -u scripts/resync_bench.py > $O/resync.txt 2>&1 &&
timeout -k 10 400 python -u scripts/dropin_bench.py > $O/dropin.txt 2>&1 &&
timeout -k 10 300 python -u scripts/adaptor_bench.py --cpu > $O/adaptor.txt 2>&1 &&
timeout -k 10 300 python -u scripts/long_unit_bench.py --auto > $O/long_unit.txt 2>&1 &&
timeout -k 10 120 python -u scripts/msg_bench.py > $O/msg_bench.txt 2>&1 &&
timeout -k 10 120 python -u scripts/percall_bench.py > $O/percall.txt 2>&1 && echo part3 done
fi
