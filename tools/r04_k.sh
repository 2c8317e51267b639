#!/bin/bash
# r04 session K: low-register P1 scatter (co-resident sort) + bucket-reduction knobs
set -e
OUT=gpurun_out/r04k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/mb_fp64 > $OUT/mb_fp64.log 2>&1
ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_msm_ntt.py -k "table or msm" > $OUT/pytest_lr.log 2>&1
REPS=2 bash tools/env_ab.sh r04k "base|X=0" "lr|ZKMI_RS_T1=2" "lr_p2|ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256" \
  "strip4|ZKMI_BR_STRIP=4" "seg64|ZKMI_BR_SEG=64" "lr_p2_l4|ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256 LANES=4"
ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_lr -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 360 --timeout-method thread tests/test_gpu_scale.py -k "2pow26_table_plan" > $OUT/pytest_26.log 2>&1
