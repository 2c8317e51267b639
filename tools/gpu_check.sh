#!/bin/bash
# Dev loop on the GPU box: the -m gpu suite, then the 2^20 table MSM at 1 and
# 3 lanes (tools/perf_table.py).  Output under gpurun_out/check/.
set -e
mkdir -p gpurun_out/check
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1
LANES=1,3 K=40 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 > gpurun_out/check/perf.log 2>&1
