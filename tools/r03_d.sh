#!/bin/bash
set -e
OUT=gpurun_out/r03d
mkdir -p $OUT
: > $OUT/sweep.log
run() { env "$@" SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 15 >> $OUT/sweep.log 2>&1; }
run SP_LANES=2
run SP_LANES=2 ZKMI_PROVE_GRAPH=1
timeout -k 10 150 python3 tools/small_prove.py 15 >> $OUT/sweep.log 2>&1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_groth16.py tests/test_gpu_l2block.py tests/test_gpu_keygen.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
