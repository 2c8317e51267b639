#!/bin/bash
# Strip bucket reduction A/B: ZKMI_BR_STRIP=8 (G1 default: one 64-lane wave per
# 512-bucket row segment or column) vs 16 (buckets per lane; 512-bucket columns
# packed two per wave, as G2 runs), 2^20 table MSM, G1 and G2.
set -e
mkdir -p gpurun_out/strip
for rep in 1 2; do
for f in 8 16; do
  if [ $f = def ]; then unset ZKMI_BR_STRIP; else export ZKMI_BR_STRIP=$f; fi
  echo "== strip $f" >> gpurun_out/strip/p.log
  LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/strip/p.log 2>&1
  LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> gpurun_out/strip/p.log 2>&1
done
done
