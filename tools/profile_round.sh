#!/bin/bash
# Bench + rocprofv3 evidence for one round (run on the GPU box via gpurun).
#   tools/profile_round.sh <tag>      -> gpurun_out/<tag>/...
# Every GPU step has its own time limit and the chain stops at the first failure.
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err
python3 tools/rocprof_summary.py $OUT/trace $OUT/bench_rocprof.json > $OUT/rocprof_summary.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py --no-plain --no-ntt --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch.json 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py --no-plain --no-ntt --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write.json 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $OUT/pmc_valu -o run -- \
    python3 bench.py --no-plain --no-ntt --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_valu.json 2>&1
python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write 20 msm_acc0_g1 $OUT/pmc_valu > $OUT/pmc_traffic.txt
cp profiles/pmc_traffic.json $OUT/
