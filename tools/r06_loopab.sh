#!/bin/bash
# headline-loop A/B over zelana_amd/_ab/libzkmi_<v>.so (VARIANTS), interleaved
set -o pipefail
OUT=gpurun_out/${TAG:-r06loop}
mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=${LANES:-2} DEPTH=${DEPTH:-2} timeout -k 10 120 python3 tools/headline_loop.py ${LOGN:-20} ${K:-60} >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
