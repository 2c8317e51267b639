# Negated-table A/B at the headline (2^20, 3 lanes, 3 interleaved repeats) and at 2^26 (2 lanes).
set -e
mkdir -p gpurun_out/neg2
for rep in 1 2 3; do
for v in 0 1; do
  echo "== neg_table $v" >> gpurun_out/neg2/p.log
  ZKMI_NEG_TABLE=$v LANES=3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/neg2/p.log 2>&1
done
done
for v in 0 1; do
  echo "== 2^26 neg_table $v" >> gpurun_out/neg2/p.log
  ZKMI_NEG_TABLE=$v LANES=2 K=8 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/neg2/p.log 2>&1
done
