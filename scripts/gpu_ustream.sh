#!/bin/bash
# Round-2 stream-unpack check: parity tests, then bench lines (stream vs tile).
set -o pipefail
TAG=${1:-us}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
for w in config2 carsales config3; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail -20 gpurun_out/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$w.json'));print('$w', {k:(v['ms'],v['frac']) for k,v in d['kernels'].items()})"
done
CAPNP_UNPACK_KERNEL=tile timeout -k 10 300 python -u bench.py --workload config2 --no-cpu > gpurun_out/${TAG}_bench_tile.json 2>&1 && python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_tile.json'));print('tile', {k:(v['ms'],v['frac']) for k,v in d['kernels'].items()})"
