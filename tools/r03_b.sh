#!/bin/bash
# Witness-program GPU tests (L2 + zelana_batch), configs[0] latency and its kernel timeline.
set -e
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_l2block.py tests/test_gpu_zbatch.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 20 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
