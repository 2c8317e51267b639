# Accumulation cost per entry vs table size (one lane, isolated kernels).
set -e
mkdir -p gpurun_out/size
for ln in 20 22 24 26; do
  echo "== $ln" >> gpurun_out/size/p.log
  K=6 LANES=1 timeout -k 10 300 python3 tools/perf_table.py $ln 0:0 >> gpurun_out/size/p.log 2>&1
done
