#!/bin/bash
# r04 session H: accumulation variants (129-VGPR one-item-per-thread, 128-capped, LDS rows, persistent)
set -e
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
S="ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256"
REPS=2 bash tools/env_ab.sh r04h "base|X=0" "base_1l|LANES=1" "base_s|$S" \
  "g128|ZKMI_LIB=zelana_amd/_ab/libzkmi_g128.so" "g128_1l|ZKMI_LIB=zelana_amd/_ab/libzkmi_g128.so LANES=1" \
  "lds|ZKMI_ACC_LDS=1" "lds_1l|ZKMI_ACC_LDS=1 LANES=1" "lds128|ZKMI_LIB=zelana_amd/_ab/libzkmi_g128.so ZKMI_ACC_LDS=1" \
  "p3_1l|ZKMI_ACC_PERS=3 LANES=1"
