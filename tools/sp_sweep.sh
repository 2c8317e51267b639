#!/bin/bash
# configs[0] resident-prove latency over table / window / lane choices (tools/small_prove.py).
set -e
OUT=gpurun_out/sp_sweep
mkdir -p $OUT
: > $OUT/sweep.log
run() { env "$@" SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 15 >> $OUT/sweep.log 2>&1; }
run SP_LANES=2
run SP_LANES=3
run ZKMI_PK_TABLE_MIN=100000 SP_LANES=2
run ZKMI_PK_TABLE_MIN=100000 SP_LANES=3
run ZKMI_PK_TABLE_MIN=100000 SP_LANES=3 SP_WINDOW=8
run ZKMI_PK_TABLE_MIN=100000 SP_LANES=3 SP_WINDOW=9
run ZKMI_TABLE_C=16 SP_LANES=3
run ZKMI_TABLE_C=10 SP_LANES=3
run ZKMI_LIB=zelana_amd/_ab/libzkmi_noasm.so SP_LANES=2
run ZKMI_LIB=zelana_amd/_ab/libzkmi_noasm.so SP_LANES=3
