# NTT A/B: in-tree build vs zelana_amd/_ab/libzkmi_<variant>.so
set -e
mkdir -p gpurun_out/ntt
for rep in 1 2 3; do
for v in base ${VARIANTS:-nttnoasm}; do
  if [ $v = base ]; then unset ZKMI_LIB; else export ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so; fi
  echo "== $v" >> gpurun_out/ntt/p.log
  timeout -k 10 120 python3 tools/perf_ntt.py 24 >> gpurun_out/ntt/p.log 2>&1
done
done
