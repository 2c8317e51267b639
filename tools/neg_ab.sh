#!/bin/bash
# Negated fixed-base table A/B: ZKMI_NEG_TABLE=1 (d_neg built, -P gathered for negative
# digits) vs the default (per-entry negation), 2^20 table MSM G1 / G2.
set -e
mkdir -p gpurun_out/neg
for rep in 1 2; do
for v in 0 1; do
  echo "== neg_table $v" >> gpurun_out/neg/p.log
  ZKMI_NEG_TABLE=$v LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/neg/p.log 2>&1
  ZKMI_NEG_TABLE=$v LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> gpurun_out/neg/p.log 2>&1
done
done
