set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_sync.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-sync > gpurun_out/b_nosync.log 2>&1
python - <<'P'
import json
for f in ("gpurun_out/b_sync.log","gpurun_out/b_nosync.log"):
    l=[x for x in open(f) if x.startswith("{")][0]; d=json.loads(l)
    print(f, d["value"], d["kernels"]["pack"]["ms"], d["kernels"]["unpack"]["ms"], d["roundtrip_ok"])
P
