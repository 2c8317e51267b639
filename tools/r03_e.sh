#!/bin/bash
set -e
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
