#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r06_l2}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 240 python3 tools/l2_loop.py 22 10 > $OUT/run.log 2>&1 || exit 1
TWO=1 timeout -k 10 240 python3 tools/l2_loop.py 22 10 >> $OUT/run.log 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o run -- python3 $GRAFT_REPO_ROOT/tools/l2_loop.py 22 4 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1
cat $GRAFT_REPO_ROOT/$OUT/run.log
