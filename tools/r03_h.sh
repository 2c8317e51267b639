#!/bin/bash
set -e
OUT=gpurun_out/r03h
mkdir -p $OUT
: > $OUT/sweep.log
run() { env "$@" SP_RESIDENT_ONLY=1 timeout -k 10 120 python3 tools/small_prove.py 20 >> $OUT/sweep.log 2>&1; }
run SP_LANES=2
run SP_LANES=3
run SP_LANES=2
run SP_LANES=3
