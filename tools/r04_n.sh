#!/bin/bash
# r04 session N: small-MSM item path + cleanup: GPU tests of the touched paths, configs[0] timing, headline
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py tests/test_gpu_groth16.py \
  tests/test_gpu_l2block.py tests/test_gpu_zbatch.py > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
REPS=2 bash tools/env_ab.sh r04n "base|X=0"
