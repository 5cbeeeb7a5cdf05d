#!/bin/bash
# GPU tests, smoke, then bench lines for the lean pack kernel and the old one (A/B).
set -o pipefail
T=${1:-r03b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
for v in 1 0 1 0; do
  CAPNP_PACK_LEAN=$v timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench_lean$v.json 2> gpurun_out/${T}_bench_lean$v.err \
    || { tail -20 gpurun_out/${T}_bench_lean$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_lean$v.json')); k=d['kernels']; print('lean=$v', d['value'], 'pack', k['pack']['ms'], 'unpack', k['unpack']['ms'], 'nosync', k['unpack_nosync']['ms'], d['roundtrip_ok'])"
done
