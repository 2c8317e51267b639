set -e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l2prof -o run -- python3 tools/perf_l2.py 22 > gpurun_out/l2prof.log 2>&1
