#!/bin/bash
set -e
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_msm_ntt.py tests/test_gpu_groth16.py tests/test_gpu_l2block.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 20 > $OUT/sweep.log 2>&1
