#!/bin/bash
# MSM A/B over zelana_amd/_ab/libzkmi_<variant>.so builds (tools/build_ab.sh):
# 2^20 table MSM, G1 at 1 and 3 lanes and G2 at 2 lanes, interleaved repeats.
#   VARIANTS="cur brgen" tools/msm_ab.sh
set -e
mkdir -p gpurun_out/msmab
for rep in 1 2; do
for v in ${VARIANTS:-cur}; do
  echo "== $v G1" >> gpurun_out/msmab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/msmab/p.log 2>&1
  echo "== $v G2" >> gpurun_out/msmab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> gpurun_out/msmab/p.log 2>&1
done
done
