#!/bin/bash
# r04 session G: accumulation at 129 (one item per thread) / 113 VGPRs (persistent, LDS rows)
set -e
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp
S="ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_scale.py -k "table_plan" > $OUT/pytest.log 2>&1
ZKMI_ACC_PERS=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_scale.py -k "table_plan" > $OUT/pytest_pers.log 2>&1
REPS=2 bash tools/env_ab.sh r04g "base|X=0" "base_1l|LANES=1" \
  "p3|ZKMI_ACC_PERS=3 $S" "p3br|ZKMI_LIB=zelana_amd/_ab/libzkmi_co2.so ZKMI_ACC_PERS=3 $S" \
  "p3_1l|ZKMI_ACC_PERS=3 LANES=1" "p4_1l|ZKMI_ACC_PERS=4 LANES=1" "p3br_2l|ZKMI_LIB=zelana_amd/_ab/libzkmi_co2.so ZKMI_ACC_PERS=3 $S LANES=2"
env ZKMI_LIB=zelana_amd/_ab/libzkmi_co2.so ZKMI_ACC_PERS=3 $S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_p3br -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr.log 2>&1
