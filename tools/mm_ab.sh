#!/bin/bash
# A/B of the affine + affine second bucket entry (ZK_MMADD): libzkmi_mm.so vs
# libzkmi_nommadd.so (tools/build_ab.sh nommadd -DZK_MMADD=0), G1 and G2 tables,
# interleaved repeats.
set -e
mkdir -p gpurun_out/mmab
for rep in 1 2; do
for v in mm nommadd; do
  echo "== $v G1" >> gpurun_out/mmab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/mmab/p.log 2>&1
  echo "== $v G2" >> gpurun_out/mmab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> gpurun_out/mmab/p.log 2>&1
done
done
