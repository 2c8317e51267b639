# Radix-sort scatter geometry A/B (ZKMI_RS_T1 / _T2 / _ST2): correctness, then
# the 2^20 table MSM (one lane: sort time; 3 lanes: rate) and 2^26 (2 lanes).
set -e
mkdir -p gpurun_out/rs
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py > gpurun_out/rs/t.log 2>&1
for cfg in "ZKMI_RS_T1=256" "ZKMI_RS_T1=1024" "ZKMI_RS_T2=1024 ZKMI_RS_ST2=4096" "ZKMI_RS_T2=1024 ZKMI_RS_ST2=8192" "ZKMI_RS_T2=1024 ZKMI_RS_ST2=16384"; do
  echo "== $cfg" >> gpurun_out/rs/p.log
  env $cfg LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/rs/p.log 2>&1
done
for cfg in "ZKMI_RS_T1=256" "ZKMI_RS_T1=1024" "ZKMI_RS_T2=1024 ZKMI_RS_ST2=8192"; do
  echo "== 26 $cfg" >> gpurun_out/rs/p.log
  env $cfg K=6 LANES=1,2 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/rs/p.log 2>&1
done
