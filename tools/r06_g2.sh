#!/bin/bash
# round 6: full GPU suite on the current tree, then headline-loop A/B of the
# saved baseline library (zelana_amd/_ab/libzkmi_base.so) against the tree's
set -o pipefail
OUT=gpurun_out/${TAG:-r06b}
mkdir -p $OUT
cp zelana_amd/libzkmi.so zelana_amd/_ab/libzkmi_cur.so
for rep in 1 2 3; do
  for v in base cur; do
    for d in 2 4; do
      echo "== $v depth $d rep $rep" >> $OUT/ab.log
      ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=$d timeout -k 10 120 python3 tools/headline_loop.py 20 60 >> $OUT/ab.log 2>&1 || exit 1
    done
  done
done
cat $OUT/ab.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
