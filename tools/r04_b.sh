#!/bin/bash
# r04 session B: persistent-accumulation A/B, mat-vec tests + configs[0] timing.
set -e
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_groth16.py \
  tests/test_gpu_l2block.py tests/test_gpu_zbatch.py > $OUT/pytest.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
REPS=2 bash tools/env_ab.sh r04b "base|X=0" "p3|ZKMI_ACC_PERS=3" "p2|ZKMI_ACC_PERS=2" "p2t|ZKMI_ACC_PERS=2 ZKMI_RS_T1=256" \
  "p2t2l|ZKMI_ACC_PERS=2 ZKMI_RS_T1=256 LANES=2" "p2t4l|ZKMI_ACC_PERS=2 ZKMI_RS_T1=256 LANES=4"
ZKMI_ACC_PERS=2 ZKMI_RS_T1=256 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_p2t -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr_p2t.log 2>&1
