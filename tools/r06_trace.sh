#!/bin/bash
# kernel trace of the 2-lane headline loop (tools/headline_loop.py) for tools/acc_gaps.py
set -o pipefail
OUT=gpurun_out/${TAG:-r06tr}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
LANES=${LANES:-2} DEPTH=${DEPTH:-4} timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o run -- python3 $GRAFT_REPO_ROOT/tools/headline_loop.py 20 30 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1
