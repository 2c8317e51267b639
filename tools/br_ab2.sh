# Interleaved repeats of the pipelined 2^20 table MSM per bucket-reduction setting.
set -e
mkdir -p gpurun_out/br2
for rep in 1 2 3; do
for cfg in "ZKMI_BR_MODE=1" "ZKMI_BR_FOLD=8" "ZKMI_BR_FOLD=8 ZKMI_BR_SEG=128" "ZKMI_BR_FOLD=4 ZKMI_BR_SEG=128"; do
  echo "== $cfg" >> gpurun_out/br2/p.log
  env $cfg LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/br2/p.log 2>&1
done
done
