#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r06_26ab}
mkdir -p $OUT
for rep in 1 2; do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=2 WARM=3 timeout -k 10 240 python3 tools/headline_loop.py 26 8 >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
