#!/bin/bash
# Round-3 final measurement set, part C: the §8(f) rows' own benches
# (message batches, flat framing, index-free resync, stream adaptors).
set -o pipefail
T=${1:-r03fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in msg_bench flat_bench resync_bench adaptor_bench; do
  timeout -k 10 300 python -u scripts/$b.py > gpurun_out/${T}_$b.txt 2> gpurun_out/${T}_$b.err \
    || { tail -20 gpurun_out/${T}_$b.err; exit 1; }
  echo "== $b"; cat gpurun_out/${T}_$b.txt
done
