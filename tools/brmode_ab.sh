# Bucket-reduction mode A/B (ZKMI_BR_MODE 0 = strip, 2 = fold + lines) on the 2^20 table MSM, G1 and G2.
set -e
mkdir -p gpurun_out/brmode
for rep in 1 2; do
for m in 0 2; do
  echo "== mode $m" >> gpurun_out/brmode/p.log
  ZKMI_BR_MODE=$m LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/brmode/p.log 2>&1
  ZKMI_BR_MODE=$m LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 g2 >> gpurun_out/brmode/p.log 2>&1
done
done
