#!/bin/bash
# A/B pack timing of the product library vs build/abl variants on several workloads
for wl in ${WLS:-config2 config3 config4 carsales}; do
  echo "== $wl"
  WL=$wl timeout -k 10 200 python scripts/wt_ablate.py || exit 1
done
