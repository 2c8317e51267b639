# No-table 2^20 MSM (c = 16): P1 scatter threads A/B.
set -e
mkdir -p gpurun_out/plain
for rep in 1 2; do
for cfg in "ZKMI_RS_T1=256" "ZKMI_RS_T1=1024"; do
  echo "== $cfg" >> gpurun_out/plain/p.log
  env $cfg LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 plain >> gpurun_out/plain/p.log 2>&1
done
done
