#!/bin/bash
# r04 session F: LDS-prefetch persistent accumulation (128 VGPRs, 3 waves/SIMD) with co-resident tails
set -e
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
S="ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256"
REPS=2 bash tools/env_ab.sh r04f "base|X=0" \
  "l128|ZKMI_LIB=zelana_amd/_ab/libzkmi_cur.so ZKMI_ACC_PERS=3 $S" \
  "l128br|ZKMI_LIB=zelana_amd/_ab/libzkmi_co2.so ZKMI_ACC_PERS=3 $S" \
  "l145|ZKMI_LIB=zelana_amd/_ab/libzkmi_l145.so ZKMI_ACC_PERS=3" \
  "l128_1lane|ZKMI_LIB=zelana_amd/_ab/libzkmi_cur.so ZKMI_ACC_PERS=3 LANES=1" \
  "base_1lane|LANES=1"
env ZKMI_LIB=zelana_amd/_ab/libzkmi_co2.so ZKMI_ACC_PERS=3 $S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_l128br -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr.log 2>&1
