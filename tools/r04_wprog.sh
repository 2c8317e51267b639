#!/bin/bash
# L2 witness-program session: its GPU tests, configs[0] latency, and a kernel
# trace of tools/small_prove.py (k_wprog_level durations vs the previous trace).
set -e
OUT=gpurun_out/${1:-r04wprog}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_l2block.py tests/test_gpu_zbatch.py > $OUT/pytest.log 2>&1
timeout -k 10 200 python3 tools/small_prove.py 10 > $OUT/small.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
