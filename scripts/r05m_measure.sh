set -o pipefail
mkdir -p gpurun_out/r05m
O=gpurun_out/r05m
timeout -k 10 300 python bench.py > $O/config2.json 2>$O/config2.err && echo c2 $(python scripts/bench_summary.py c2 $O/config2.json) &&
for w in config3 carsales config4; do timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/$w.json 2>/dev/null && python scripts/bench_summary.py $w $O/$w.json || exit 1; done &&
timeout -k 10 300 python bench.py --workload config3 --chunks 23400000 --steps 5 --warmup 1 --no-cpu > $O/config3_full.json 2>/dev/null && python scripts/bench_summary.py c3full $O/config3_full.json &&
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $O/config5.json 2>/dev/null && python scripts/bench_summary.py c5 $O/config5.json &&
timeout -k 10 300 python -u scripts/stream_bench.py > $O/stream.json 2>/dev/null && tail -c 600 $O/stream.json &&
timeout -k 10 300 python -u scripts/resync_bench.py > $O/resync.txt 2>&1 && tail -12 $O/resync.txt &&
timeout -k 10 400 python -u scripts/dropin_bench.py > $O/dropin.txt 2>&1 && head -3 $O/dropin.txt
