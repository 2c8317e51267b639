#!/bin/bash
# Round-3 first GPU pass: the -m gpu suite, then configs[0] latency.
set -e
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 20 > $OUT/small.log 2>&1
