#!/bin/bash
# Headline-loop A/B over zelana_amd/_ab/libzkmi_<variant>.so (tools/build_ab.sh),
# interleaved repeats, timers off.   VARIANTS="cur p0" REPS=3 tools/loop_ab.sh <tag>
set -e
OUT=gpurun_out/${1:-loopab}
mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-cur}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=${LANES:-3} timeout -k 10 120 python3 tools/headline_loop.py ${LOGN:-20} ${K:-40} >> $OUT/ab.log 2>&1
  done
done
if [ -n "$TRACE" ]; then
  export TMPDIR=/tmp
  for v in $TRACE; do
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$v -o run -- python3 tools/headline_loop.py 20 30 > $OUT/tr_$v.log 2>&1
  done
fi
