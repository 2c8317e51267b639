#!/bin/bash
set -e
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 > $OUT/perf.log 2>&1
LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> $OUT/perf.log 2>&1
SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 15 >> $OUT/perf.log 2>&1
VARIANTS=frc timeout -k 10 400 bash tools/ntt_ab.sh
