#!/bin/bash
# Round-4 evidence from the final tree (run via gpurun): the GPU suite, the
# bench line + rocprofv3 stats + PMC passes (tools/profile_r02.sh), a kernel
# trace of the 3-lane headline loop (accumulation-idle fraction,
# tools/acc_gaps.py) and of the configs[0] resident proof (tools/trace_proof.py).
set -e
TAG=${1:-r04final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1
fi
bash tools/profile_r02.sh $TAG
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/loop3 -o run -- python3 tools/headline_loop.py 20 30 > $OUT/loop3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small -o run -- python3 tools/small_prove.py 5 > $OUT/small.log 2>&1
