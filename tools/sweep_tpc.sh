set -e
for t in 768 1024 2048 4096 8192; do
  echo "== tpc $t"
  ZKMI_ACC_TPC=$t LANES=1 timeout -k 10 120 python3 tools/perf_table.py 20 17:0 | grep -E "acc0|accN|pipelined"
  ZKMI_ACC_TPC=$t LANES=1 timeout -k 10 120 python3 tools/perf_table.py 18 17:0 g2 | grep -E "acc0|accN|pipelined"
done
