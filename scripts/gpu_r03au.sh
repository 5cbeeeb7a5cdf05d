#!/bin/bash
# Config 3 at the SURVEY's full size (23.4 M x 1 KiB, 4 GiB packed) and one
# config-5 shard (8 Mi x 1 KiB = 8 GiB) on the final library.
set -o pipefail
T=${1:-r03au}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --workload config3 --chunks 23400000 --steps 5 --warmup 1 --no-cpu \
  > gpurun_out/${T}_config3_full_bench.json 2> gpurun_out/${T}_config3_full.err \
  || { tail -20 gpurun_out/${T}_config3_full.err; exit 1; }
python scripts/bench_summary.py config3_full gpurun_out/${T}_config3_full_bench.json
timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu \
  > gpurun_out/${T}_config5_bench.json 2> gpurun_out/${T}_config5.err \
  || { tail -20 gpurun_out/${T}_config5.err; exit 1; }
python scripts/bench_summary.py config5 gpurun_out/${T}_config5_bench.json
