#!/bin/bash
# Round-2 evidence on the GPU box (run via gpurun): the bench line, a
# rocprofv3 kernel trace of the same command, and separate PMC passes (one
# counter group each, MI355X_MICROARCH.md) over a short bench run.
#   tools/profile_r02.sh <tag>   -> gpurun_out/<tag>/...
set -e
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err
SHORT="--no-plain --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py $SHORT > $OUT/pmc_fetch.json 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py $SHORT > $OUT/pmc_write.json 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc_valu -o run -- python3 bench.py $SHORT > $OUT/pmc_valu.json 2>&1
python3 tools/pmc_r02.py $OUT > $OUT/pmc_summary.txt
