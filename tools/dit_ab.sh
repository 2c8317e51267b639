#!/bin/bash
# NTT A/B incl. the DIT passes of the witness map: 2^24 NTT+INTT (DIF passes)
# and the 2^22 Groth16 prove's ntt_group stage at one lane (tools/perf_l2.py),
# in-tree build vs zelana_amd/_ab/libzkmi_<variant>.so, interleaved.
set -e
mkdir -p gpurun_out/dit
for rep in 1 2; do
for v in base ${VARIANTS:-nttdif nttold}; do
  if [ $v = base ]; then unset ZKMI_LIB; else export ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so; fi
  echo "== $v" >> gpurun_out/dit/p.log
  timeout -k 10 120 python3 tools/perf_ntt.py 24 >> gpurun_out/dit/p.log 2>&1
  timeout -k 10 200 python3 tools/perf_l2.py 22 >> gpurun_out/dit/p.log 2>&1
done
done
