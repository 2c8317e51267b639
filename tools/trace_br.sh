#!/bin/bash
# Kernel trace of the 2^20 table MSM at one lane under bucket-reduction modes
# (ZKMI_BR_MODE / ZKMI_BR_FOLD), for per-kernel durations.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trbr
for m in ${MODES:-1 2:4 2:8}; do
  mode=${m%%:*}; fold=${m#*:}; [ "$fold" = "$m" ] && fold=8
  ZKMI_BR_MODE=$mode ZKMI_BR_FOLD=$fold LANES=1 K=10 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trbr/m$mode.$fold -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/trbr/m$mode.$fold.log 2>&1
done
