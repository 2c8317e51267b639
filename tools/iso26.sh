# 2^26 table MSM (c = 22, 12 copies): one-lane kernel trace, then 2 lanes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/iso26
LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/iso26/p -o run -- python3 tools/perf_table.py 26 0:0 > gpurun_out/iso26/p.log 2>&1
LANES=2 timeout -k 10 300 python3 tools/perf_table.py 26 0:0 >> gpurun_out/iso26/p.log 2>&1
