# Clean per-kernel times of the headline 2^20 table MSM (one lane, serial),
# then the pipelined rate at 1..3 lanes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/iso
LANES=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/iso/p -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/iso/p.log 2>&1
LANES=1,2,3 timeout -k 10 150 python3 tools/perf_table.py 20 0:0 >> gpurun_out/iso/p.log 2>&1
