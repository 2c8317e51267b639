#!/bin/bash
set -e
OUT=gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
