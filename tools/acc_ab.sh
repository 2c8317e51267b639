#!/bin/bash
# Accumulation-kernel A/B over zelana_amd/_ab/libzkmi_<variant>.so builds
# (tools/build_ab.sh): 2^20 G1 table MSM at 1 and 3 lanes, interleaved repeats.
#   VARIANTS="v1 cur" tools/acc_ab.sh
set -e
mkdir -p gpurun_out/accab
for rep in 1 2 3; do
for v in ${VARIANTS:-cur}; do
  echo "== $v" >> gpurun_out/accab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=1,3 K=40 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 2>&1 | grep -E "pipelined|acc0" >> gpurun_out/accab/p.log
done
done
