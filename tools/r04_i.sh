#!/bin/bash
# r04 session I: persistent accumulation, one 768-thread workgroup per CU (3 waves/SIMD)
set -e
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
S="ZKMI_RS_T1=256 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256"
ZKMI_ACC_PERS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_scale.py -k "table_plan" > $OUT/pytest_pers.log 2>&1
REPS=2 bash tools/env_ab.sh r04i "base|X=0" "base_1l|LANES=1" "p1|ZKMI_ACC_PERS=1" "p1s|ZKMI_ACC_PERS=1 $S" \
  "p1_1l|ZKMI_ACC_PERS=1 LANES=1" "p1s_2l|ZKMI_ACC_PERS=1 $S LANES=2" "p1t1|ZKMI_ACC_PERS=1 ZKMI_RS_T1=256"
env ZKMI_ACC_PERS=1 $S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_p1s -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr.log 2>&1
