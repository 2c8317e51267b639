#!/bin/bash
# kernel trace of resident configs[0] proofs (tools/small_prove.py, resident only)
set -o pipefail
OUT=gpurun_out/${TAG:-r06small_tr}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
SP_RESIDENT_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/tr -o run -- python3 $R/tools/small_prove.py 10 > $R/$OUT/run.log 2>&1 || exit 1
grep resident_ms $R/$OUT/run.log
