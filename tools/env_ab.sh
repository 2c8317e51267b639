#!/bin/bash
# Headline-loop A/B over environment settings, interleaved repeats, timers off.
#   tools/env_ab.sh <tag> "name1|VAR=a VAR2=b" "name2|VAR=c" ...    (REPS, LOGN, K, LIB)
set -e
OUT=gpurun_out/${1:-envab}
shift
mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do
  for cfg in "$@"; do
    name=${cfg%%|*}
    envs=${cfg#*|}
    echo "== $name rep $rep ($envs)" >> $OUT/ab.log
    env $envs timeout -k 10 120 python3 tools/headline_loop.py ${LOGN:-20} ${K:-40} >> $OUT/ab.log 2>&1
  done
done
