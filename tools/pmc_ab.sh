# A/B PMC comparison of MSM accumulation variants (dev tool; run via gpurun)
#   VARIANTS="name=lib.so[:kernel] ..."   (lib "" = in-tree build)
#   LOGN, CFG, CURVE (g1|g2) select the perf_table.py workload
set -e
export TMPDIR=/tmp
for spec in $VARIANTS; do
  V=${spec%%=*}; rest=${spec#*=}; L=${rest%%:*}; K=k_msm_acc0_${CURVE:-g1}
  [ "$rest" != "$L" ] && K=${rest#*:}
  if [ -n "$L" ]; then export ZKMI_LIB=$L; else unset ZKMI_LIB; fi
  LANES=1 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc$V -o run -- python3 tools/perf_table.py ${LOGN:-20} ${CFG:-17:0} ${CURVE:-g1} > gpurun_out/pmc$V.log 2>&1
  python3 tools/pmc_kernel.py gpurun_out/pmc$V "$K" > gpurun_out/pmc$V.txt
done
