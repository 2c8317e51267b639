#!/bin/bash
# End-of-round evidence: bench + rocprofv3 + PMC (tools/profile_r02.sh), then
# the configs[0] timeline.
set -e
bash tools/profile_r02.sh r03final2
OUT=gpurun_out/r03final2
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small_trace -o run -- python3 tools/small_prove.py 5 > $OUT/small_prof.log 2>&1
