#!/bin/bash
# Accumulation-chain confirmation: the GPU suite, then the bench's MSM and
# proof legs, interleaved with zelana_amd/_ab/libzkmi_prev.so.
set -e
TAG=${1:-r04chain3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1
SHORT="--no-plain --no-big --no-ntt --no-cpu-baseline"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $SHORT > $OUT/bench_cur$rep.json 2> $OUT/bench_cur$rep.err
  ZKMI_LIB=zelana_amd/_ab/libzkmi_prev.so timeout -k 10 300 python3 bench.py $SHORT > $OUT/bench_prev$rep.json 2> $OUT/bench_prev$rep.err
done
