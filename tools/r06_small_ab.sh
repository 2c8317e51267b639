#!/bin/bash
# configs[0] latency A/B over zelana_amd/_ab/libzkmi_<v>.so (VARIANTS): parity
# tests of each variant in VTEST, then tools/small_prove.py interleaved
set -o pipefail
OUT=gpurun_out/${TAG:-r06small}
mkdir -p $OUT
for v in ${VTEST:-}; do
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu ${TESTS:-tests/test_gpu_msm_ntt.py tests/test_gpu_groth16.py} > $OUT/tests_$v.log 2>&1 || { tail -n 20 $OUT/tests_$v.log; exit 1; }
  tail -n 1 $OUT/tests_$v.log
done
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 200 python3 tools/small_prove.py 40 >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
