# Bit-sum segment length (ZKMI_BR_SEG) with the strip reduction, 2^20 table MSM.
set -e
mkdir -p gpurun_out/seg
for rep in 1 2; do
for cfg in "ZKMI_BR_SEG=256" "ZKMI_BR_SEG=128" "ZKMI_BR_SEG=64"; do
  echo "== $cfg" >> gpurun_out/seg/p.log
  env $cfg LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/seg/p.log 2>&1
done
done
