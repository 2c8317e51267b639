#!/bin/bash
# MSM variant check + A/B: parity tests of each variant in VTEST (if any),
# then the 2^20 headline loop and the 2^26 loop over VARIANTS, interleaved
set -o pipefail
OUT=gpurun_out/${TAG:-r06msm}
mkdir -p $OUT
for v in ${VTEST:-}; do
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu tests/test_gpu_msm_ntt.py tests/test_gpu_scale.py -k "msm or 2pow26 or table or sort" > $OUT/tests_$v.log 2>&1 || { tail -n 20 $OUT/tests_$v.log; exit 1; }
  tail -n 1 $OUT/tests_$v.log
done
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=2 timeout -k 10 120 python3 tools/headline_loop.py 20 60 >> $OUT/ab.log 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=2 WARM=3 timeout -k 10 240 python3 tools/headline_loop.py 26 8 >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
