#!/bin/bash
# r04 session C: mat-vec (host-binned long rows) tests + configs[0] timing;
# headline floor without tails (ZKMI_DEBUG_SKIP, timing only), table window A/B.
set -e
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_groth16.py \
  tests/test_gpu_l2block.py tests/test_gpu_zbatch.py > $OUT/pytest.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
REPS=2 bash tools/env_ab.sh r04c "base|X=0" "skip1|ZKMI_DEBUG_SKIP=1" "skip4|ZKMI_DEBUG_SKIP=4" "skip5|ZKMI_DEBUG_SKIP=5" \
  "c19|ZKMI_TABLE_C=19" "c21|ZKMI_TABLE_C=21" "d4|DEPTH=4"
ZKMI_DEBUG_SKIP=5 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_skip5 -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr_skip5.log 2>&1
