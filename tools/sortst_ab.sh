# High-priority shared sort stream (ZKMI_SORT_STREAM) A/B: correctness, then
# the 2^26 table MSM at 2 lanes and the 2^20 one at 3 lanes.
set -e
mkdir -p gpurun_out/sst
ZKMI_SORT_STREAM=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py > gpurun_out/sst/t.log 2>&1
for rep in 1 2; do
for v in 0 1; do
  echo "== 26 SORT_STREAM=$v" >> gpurun_out/sst/p.log
  ZKMI_SORT_STREAM=$v K=8 LANES=2 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/sst/p.log 2>&1
  echo "== 20 SORT_STREAM=$v" >> gpurun_out/sst/p.log
  ZKMI_SORT_STREAM=$v LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/sst/p.log 2>&1
done
done
