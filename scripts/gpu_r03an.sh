#!/bin/bash
# Diagnostics for round 4 on the final tree: unpack phase timelines (with and
# without the index), smoke(), one more default bench line.
set -o pipefail
T=${1:-r03an}
mkdir -p gpurun_out
export TMPDIR=/tmp
A=capnproto-rust_amd/build/abl
timeout -k 10 120 python -u scripts/unpack_prof.py --sync --lib $A/libcapnp_packed_uprof.so > gpurun_out/${T}_uprof_sync.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_uprof_sync.txt; exit 1; }
echo "== uprof sync"; grep -v amdgpu.ids gpurun_out/${T}_uprof_sync.txt
timeout -k 10 120 python -u scripts/unpack_prof.py --lib $A/libcapnp_packed_uprof.so > gpurun_out/${T}_uprof_nosync.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_uprof_nosync.txt; exit 1; }
echo "== uprof nosync"; grep -v amdgpu.ids gpurun_out/${T}_uprof_nosync.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -2 gpurun_out/${T}_smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python scripts/bench_summary.py default gpurun_out/${T}_bench.json
