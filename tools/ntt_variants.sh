#!/bin/bash
# NTT A/B over built libraries (in-tree "cur" + zelana_amd/_ab/libzkmi_<v>.so):
# interleaved perf_ntt timings and one kernel trace per variant (per-pass
# durations: python3 tools/ntt_passes.py gpurun_out/<tag>).
#   tools/ntt_variants.sh <tag> v1 v2 ...
set -e
OUT=gpurun_out/${1:-nttv}
shift
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset ZKMI_LIB; else export ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so; fi
    echo "== $v" >> $OUT/perf.log
    timeout -k 10 120 python3 tools/perf_ntt.py 24 22 >> $OUT/perf.log 2>&1
  done
done
for v in cur "$@"; do
  if [ $v = cur ]; then unset ZKMI_LIB; else export ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$v -o run -- python3 tools/perf_ntt.py 24 22 > $OUT/tr_$v.log 2>&1
done
