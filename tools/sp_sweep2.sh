#!/bin/bash
set -e
OUT=gpurun_out/sp_sweep
mkdir -p $OUT
: > $OUT/sweep2.log
run() { env "$@" SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 15 >> $OUT/sweep2.log 2>&1; }
run SP_LANES=2
run ZKMI_LIB=zelana_amd/_ab/libzkmi_noasm.so SP_LANES=2
run ZKMI_LIB=zelana_amd/_ab/libzkmi_noasm.so SP_LANES=3
run ZKMI_LIB=zelana_amd/_ab/libzkmi_noasm.so SP_LANES=2 ZKMI_TABLE_C=10
