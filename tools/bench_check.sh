#!/bin/bash
# Full 1-GPU bench line, then a 2-rank gloo rehearsal of the N > 1 path on the
# same GPU (no CPU legs).  Output under gpurun_out/bench/.
set -e
mkdir -p gpurun_out/bench
timeout -k 10 560 python3 -u bench.py > gpurun_out/bench/n1.log 2>&1
ZKMI_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline --no-zbatch \
  --no-l2 > gpurun_out/bench/n2_gloo.log 2>&1
