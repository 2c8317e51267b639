# Accumulation-kernel occupancy A/B (tools/build_ab.sh variants).
set -e
mkdir -p gpurun_out/occab
for rep in 1 2; do
for v in ${VARIANTS:-base g4 g1}; do
  echo "== $v" >> gpurun_out/occab/p.log
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/occab/p.log 2>&1
done
done
