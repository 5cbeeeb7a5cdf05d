set -o pipefail
# round-5 closing measurements (after the per-call work): tests, smoke, every workload line,
# config-2 kernel stats, the drop-in and adaptor benches
O=${OUTDIR:-gpurun_out/r05y}
mkdir -p $O
PART=${1:-1}
if [ "$PART" = 1 ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && tail -1 $O/smoke.txt &&
timeout -k 10 300 python bench.py > $O/config2.json 2>$O/config2.err && python scripts/bench_summary.py c2 $O/config2.json &&
for w in config3 carsales config4; do timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/$w.json 2>/dev/null && python scripts/bench_summary.py $w $O/$w.json || exit 1; done &&
timeout -k 10 300 python bench.py --workload config3 --chunks 23400000 --steps 5 --warmup 1 --no-cpu > $O/config3_full.json 2>/dev/null && python scripts/bench_summary.py c3full $O/config3_full.json &&
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $O/config5.json 2>/dev/null && python scripts/bench_summary.py c5 $O/config5.json && echo part1 done
else
bash scripts/traffic.sh $O/tr_c2 > $O/tr_c2.txt 2>&1 &&
bash scripts/traffic.sh $O/tr_c4 --workload config4 --steps 3 --warmup 1 --no-cpu > $O/tr_c4.txt 2>&1 &&
timeout -k 10 300 python -u scripts/stream_bench.py > $O/stream.json 2>/dev/null &&
timeout -k 10 300 python -u scripts/resync_bench.py > $O/resync.txt 2>&1 &&
timeout -k 10 400 python -u scripts/dropin_bench.py > $O/dropin.txt 2>&1 &&
timeout -k 10 300 python -u scripts/adaptor_bench.py > $O/adaptor.txt 2>&1 &&
timeout -k 10 120 python -u scripts/msg_bench.py > $O/msg_bench.txt 2>&1 &&
timeout -k 10 120 python -u scripts/percall_bench.py > $O/percall.txt 2>&1 && echo done
fi
