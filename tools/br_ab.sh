# Bucket-reduction A/B on the 2^20 table MSM: correctness tests, then the
# pipelined rate per ZKMI_BR_* setting and a one-lane kernel trace.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/br
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py -k "table or items or shared or sharded" > gpurun_out/br/t.log 2>&1
for cfg in "ZKMI_BR_MODE=1" "ZKMI_BR_FOLD=4" "ZKMI_BR_FOLD=8" "ZKMI_BR_SEG=128" "ZKMI_BR_SEG=256"; do
  echo "== $cfg" >> gpurun_out/br/p.log
  env $cfg LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/br/p.log 2>&1
done
LANES=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/br/prof -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/br/prof.log 2>&1
