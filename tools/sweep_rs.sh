#!/bin/bash
# Dev sweep (GPU box): radix-sort geometry (ZKMI_RS_LOB / ZKMI_RS_C2 / ZKMI_RS_ST1 / ZKMI_RS_ST2) at 2^20 and 2^26, one lane.
#   tools/sweep_rs.sh <outdir> "<lob:c2[:st1:st2]> ..." [logn...]
OUT=$1; CFGS=$2; shift 2
mkdir -p $OUT
for ln in ${@:-20 26}; do
  for cfg in $CFGS; do
    IFS=: read lob c2 st1 st2 <<< "$cfg"
    echo "== 2^$ln lob=$lob c2=$c2 st1=${st1:-4096} st2=${st2:-4096}" >> $OUT/sweep.txt
    ZKMI_RS_LOB=$lob ZKMI_RS_C2=$c2 ZKMI_RS_ST1=${st1:-4096} ZKMI_RS_ST2=${st2:-4096} LANES=1 timeout -k 10 120 python3 tools/perf_table.py $ln 20:0 >> $OUT/sweep.txt 2>&1 || exit 1
  done
done
