#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r06ntt}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 120 python3 tools/ntt_loop.py 24 20 >> $OUT/ab.log 2>&1 || exit 1
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 120 python3 tools/ntt_loop.py 22 40 >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
