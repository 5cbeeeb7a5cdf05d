#!/bin/bash
# rocprofv3 kernel stats of one command: scripts/prof_cmd.sh <tag> <cmd...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- "$@" \
  > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(5), "%10.1f us" % (float(r['AverageNs'])/1e3))
PY
