#!/bin/bash
# 2^26 table MSM loop (c = 22, 12 copies): lanes / depth A/B and a kernel trace
set -o pipefail
OUT=gpurun_out/${TAG:-r06_26}
mkdir -p $OUT
for cfg in "2 2" "2 3" "3 3"; do
  set -- $cfg
  echo "== lanes $1 depth $2" >> $OUT/ab.log
  LANES=$1 DEPTH=$2 WARM=3 timeout -k 10 240 python3 tools/headline_loop.py 26 8 >> $OUT/ab.log 2>&1 || exit 1
done
export TMPDIR=/tmp
cd /tmp
LANES=2 DEPTH=2 WARM=3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o run -- python3 $GRAFT_REPO_ROOT/tools/headline_loop.py 26 6 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1
cat $GRAFT_REPO_ROOT/$OUT/ab.log
