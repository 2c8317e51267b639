#!/bin/bash
# the round-end GPU checks on the current tree: pytest -m gpu (as the driver
# runs it) and __graft_entry__.smoke()
set -o pipefail
OUT=gpurun_out/${TAG:-r06suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -2 $OUT/smoke.log
exit $rc
