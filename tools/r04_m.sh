#!/bin/bash
# r04 session M: full GPU suite after the knob cleanup, FP64 microbench, co-resident sort A/B
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/mb_fp64 > $OUT/mb_fp64.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || exit 1
REPS=2 bash tools/env_ab.sh r04m "base|X=0" "lr|ZKMI_RS_T1=2" "lr_p2|ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256" \
  "lr_p2_l4|ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256 LANES=4"
ZKMI_RS_T1=2 ZKMI_RS_ST2=4096 ZKMI_RS_T2=256 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_lr -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
