# Interleaved repeats: lanes x bucket-reduction mode on the 2^20 table MSM.
set -e
mkdir -p gpurun_out/lanes
for rep in 1 2; do
for cfg in "LANES=3 ZKMI_BR_MODE=1" "LANES=3 ZKMI_BR_MODE=2" "LANES=4 ZKMI_BR_MODE=1" "LANES=4 ZKMI_BR_MODE=2" "LANES=2 ZKMI_BR_MODE=1"; do
  echo "== $cfg" >> gpurun_out/lanes/p.log
  env $cfg timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/lanes/p.log 2>&1
done
done
