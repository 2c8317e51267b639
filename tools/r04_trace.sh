#!/bin/bash
# Kernel traces of the headline loop (3 lanes and 1 lane) for tools/acc_gaps.py.
#   tools/r04_trace.sh <tag>  -> gpurun_out/<tag>/
set -e
TAG=${1:-tr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/headline_loop.py 20 30 > $OUT/loop3.log 2>&1
LANES=1 timeout -k 10 120 python3 tools/headline_loop.py 20 30 > $OUT/loop1.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o run -- python3 tools/headline_loop.py 20 30 > $OUT/p3.log 2>&1
LANES=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 tools/headline_loop.py 20 20 > $OUT/p1.log 2>&1
