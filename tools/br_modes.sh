#!/bin/bash
# 2^20 table MSM, 1 and 3 lanes, under bucket-reduction modes (MODES="1 3:4 3:8").
set -e
mkdir -p gpurun_out/brm
for rep in 1 2; do
for m in ${MODES:-1 3:4 3:8}; do
  mode=${m%%:*}; fold=${m#*:}; [ "$fold" = "$m" ] && fold=8
  echo "== mode $mode fold $fold" >> gpurun_out/brm/p.log
  ZKMI_BR_MODE=$mode ZKMI_BR_FOLD=$fold LANES=1,3 K=40 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 2>&1 | grep -E "pipelined|bucket" >> gpurun_out/brm/p.log
done
done
