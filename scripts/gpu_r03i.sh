#!/bin/bash
# Phase timeline of the index-free unpack (UNPACK_PROF build) and the indexed one.
set -o pipefail
T=${1:-r03i}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 180 python -u scripts/unpack_prof.py > gpurun_out/${T}_uprof.txt 2>&1 || { tail -20 gpurun_out/${T}_uprof.txt; exit 1; }
cat gpurun_out/${T}_uprof.txt


