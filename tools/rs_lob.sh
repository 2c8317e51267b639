# 2^26 table MSM: P1/P2 digit split (ZKMI_RS_LOB), then the default bench.
set -e
mkdir -p gpurun_out/lob
for cfg in "ZKMI_RS_LOB=12" "ZKMI_RS_LOB=11" "ZKMI_RS_LOB=13"; do
  echo "== 26 $cfg" >> gpurun_out/lob/p.log
  env $cfg K=6 LANES=1,2 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/lob/p.log 2>&1
done
timeout -k 10 600 python3 bench.py > gpurun_out/lob/bench.json 2> gpurun_out/lob/bench.err
