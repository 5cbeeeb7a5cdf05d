#!/bin/bash
# GPU tests, smoke, then bench A/B: cs (default) / lean / old pack kernels.
set -o pipefail
T=${1:-r03c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
for rep in 1 2; do
for v in "cs" "lean CAPNP_PACK_CS=0" "old CAPNP_PACK_CS=0 CAPNP_PACK_LEAN=0"; do
  set -- $v; name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/${T}_bench_$name.json 2> gpurun_out/${T}_bench_$name.err \
    || { tail -20 gpurun_out/${T}_bench_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_$name.json')); k=d['kernels']; print('$name', d['value'], 'pack', k['pack']['ms'], 'unpack', k['unpack']['ms'], 'nosync', k['unpack_nosync']['ms'], d['roundtrip_ok'])"
done
done
