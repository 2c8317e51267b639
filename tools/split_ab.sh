# Accumulation split into k launches (ZKMI_ACC_SPLIT) A/B.
set -e
mkdir -p gpurun_out/split
ZKMI_ACC_SPLIT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm_ntt.py -k "table or items or shared" > gpurun_out/split/t.log 2>&1
for rep in 1 2; do
for k in 1 2 4; do
  echo "== 26 SPLIT=$k" >> gpurun_out/split/p.log
  ZKMI_ACC_SPLIT=$k K=8 LANES=2 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/split/p.log 2>&1
done
for k in 1 2; do
  echo "== 20 SPLIT=$k" >> gpurun_out/split/p.log
  ZKMI_ACC_SPLIT=$k LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/split/p.log 2>&1
done
done
