#!/bin/bash
# One parametrised GPU-box runner (replaces the per-run gpu_r0*.sh scripts):
#   scripts/gpu.sh TAG STEP [STEP ...]
# Each step runs under its own time limit; the first failing step ends the
# call (no GPU work after a fault, a timeout or an abort).  Outputs go to
# gpurun_out/TAG_*.
# Steps:
#   tests              pytest -m gpu over tests/
#   tests=FILE[,FILE]  pytest -m gpu over the given test files
#   smoke              __graft_entry__.smoke()
#   bench              bench.py (the driver's default line)
#   bench=W            bench.py --workload W
#   prof=W             rocprofv3 kernel trace + PMC passes of bench.py --workload W (scripts/profile.sh)
#   trace=W            rocprofv3 --kernel-trace --stats of bench.py --workload W only
#   py=SCRIPT[,ARG...] python -u scripts/SCRIPT ARG...
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/$TAG
fail() { echo "STEP FAILED: $1"; tail -40 "$2"; exit 1; }
k=0
for step in "$@"; do
  name=${step%%=*}
  arg=
  [[ $step == *=* ]] && arg=${step#*=}
  case $name in
    tests)
      tgt=tests
      [ -n "$arg" ] && tgt=$(echo "$arg" | tr ',' ' ')
      timeout -k 10 900 python -u -m pytest $tgt -m gpu -x -v --timeout 200 --timeout-method thread \
        > ${O}_tests.log 2>&1 || fail "$step" ${O}_tests.log
      tail -1 ${O}_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 \
        || fail "$step" ${O}_smoke.txt
      tail -1 ${O}_smoke.txt ;;
    bench)
      w=${arg:-default}
      wa=
      [ -n "$arg" ] && wa="--workload $arg"
      timeout -k 10 400 python -u bench.py $wa > ${O}_${w}_bench.json 2> ${O}_${w}_bench.err \
        || fail "$step" ${O}_${w}_bench.err
      python scripts/bench_summary.py $w ${O}_${w}_bench.json ;;
    prof)
      timeout -k 10 1000 bash scripts/profile.sh ${O}_prof_${arg} --workload ${arg} --steps 5 --warmup 1 --no-cpu \
        > ${O}_prof_${arg}.log 2>&1 || fail "$step" ${O}_prof_${arg}.log
      cat ${O}_prof_${arg}/summary.txt ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_trace_${arg} -o run --output-format csv \
        -- python3 bench.py --workload ${arg} --steps 20 --warmup 3 --no-cpu > ${O}_trace_${arg}.json 2> ${O}_trace_${arg}.err \
        || fail "$step" ${O}_trace_${arg}.err
      python scripts/bench_summary.py prof ${O}_trace_${arg}.json ;;
    py)
      IFS=',' read -r -a pa <<< "$arg"
      k=$((k + 1))
      f=${O}_py${k}_${pa[0]%.py}.txt
      timeout -k 10 600 python -u scripts/${pa[0]} "${pa[@]:1}" > $f 2>&1 || fail "$step" $f
      grep -v amdgpu.ids $f | tail -40 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
