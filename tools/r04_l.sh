#!/bin/bash
# r04 session L: configs[0] table-window sweep (small-MSM latency)
set -e
OUT=gpurun_out/r04l
mkdir -p $OUT
for c in 13 8 9 10 11 12 13; do
  echo "== c=$c" >> $OUT/sweep.log
  ZKMI_TABLE_C=$c timeout -k 10 120 python3 tools/small_prove.py 10 >> $OUT/sweep.log 2>&1
done
