#!/bin/bash
# Round-6 evidence from the final tree (run via gpurun): PART=A: PMC passes
# (so the bench line's roofline.traffic is this tree's) and the bench line;
# PART=B: the same bench under rocprofv3 --kernel-trace --stats, a kernel
# trace of the 2-lane headline loop (tools/acc_gaps.py), the configs[0]
# resident-proof trace and the 2-rank gloo rehearsal of the N > 1 path.
set -e
TAG=${TAG:-r06final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date >> $OUT/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
if [ "${PART:-A}" = A ]; then
SHORT="--no-plain --no-l2 --no-zbatch --no-big --no-g2 --no-window-ab --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py $SHORT > $OUT/pmc_fetch.json 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py $SHORT > $OUT/pmc_write.json 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc_valu -o run -- python3 bench.py $SHORT > $OUT/pmc_valu.json 2>&1
python3 tools/pmc_r02.py $OUT > $OUT/pmc_summary.txt
cp profiles/pmc_traffic.json $OUT/
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
else
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err
python3 tools/rocprof_summary.py $OUT/trace $OUT/bench_rocprof.json > $OUT/rocprof_summary.txt
LANES=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/loop2 -o run -- python3 tools/headline_loop.py 20 30 > $OUT/loop2.log 2>&1
python3 tools/acc_gaps.py $OUT/loop2/run_kernel_trace.csv > $OUT/headline_loop2_acc_gaps.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/small -o run -- python3 tools/small_prove.py 5 > $OUT/small.log 2>&1
ZKMI_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline --no-zbatch \
  --no-l2 > $OUT/gloo2_rehearsal.json 2> $OUT/gloo2_rehearsal.err
fi
