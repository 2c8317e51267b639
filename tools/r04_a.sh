#!/bin/bash
# r04 session A: tail-priority A/B + trace, the sharded host test, GPU tests of
# the touched paths, configs[0] latency + timeline.
set -e
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
VARIANTS="cur p0 p1" TRACE="cur p0" bash tools/loop_ab.sh r04a
timeout -k 10 180 ./zelana_amd/test_sharded_msm > $OUT/sharded.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_zbatch.py \
  tests/test_gpu_groth16.py tests/test_gpu_l2block.py > $OUT/pytest.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
