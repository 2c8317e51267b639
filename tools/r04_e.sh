#!/bin/bash
# r04 session E: co-residency A/B (acc capped at 3 waves x 128 VGPRs, tails <= 128, 256-thread sort scatters)
set -e
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
CO="ZKMI_LIB=zelana_amd/_ab/libzkmi_co.so ZKMI_ACC_PERS=3 ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256"
REPS=2 bash tools/env_ab.sh r04e "base|X=0" "co|$CO" "co_l2|$CO LANES=2" "co_l4|$CO LANES=4" \
  "cop2|ZKMI_LIB=zelana_amd/_ab/libzkmi_co.so ZKMI_ACC_PERS=2 ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256" \
  "co_t1only|ZKMI_LIB=zelana_amd/_ab/libzkmi_co.so ZKMI_ACC_PERS=3 ZKMI_RS_T1=256"
env $CO timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_co -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr_co.log 2>&1
