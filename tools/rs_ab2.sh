# Interleaved repeats, 2^20 table MSM at 3 lanes, sort geometries.
set -e
mkdir -p gpurun_out/rs2
for rep in 1 2 3; do
for cfg in "ZKMI_RS_T1=256" "ZKMI_RS_T1=1024" "ZKMI_RS_T2=1024 ZKMI_RS_ST2=8192"; do
  echo "== $cfg" >> gpurun_out/rs2/p.log
  env $cfg LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/rs2/p.log 2>&1
done
done
