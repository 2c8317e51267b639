# Attribution of the pipelined 2^20 table-MSM step: re-run with the sort +
# item plan re-used (bit 1) and / or the bucket reduction skipped (bit 4).
# Timing only (ZKMI_DEBUG_SKIP, msm.hip); the 'same=' column is meaningless
# when bit 4 is set.
set -e
mkdir -p gpurun_out/abl
for s in 0 1 4 5; do
  echo "== ZKMI_DEBUG_SKIP=$s" >> gpurun_out/abl/a.log
  ZKMI_DEBUG_SKIP=$s LANES=${LANES:-3} timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/abl/a.log 2>&1
done
