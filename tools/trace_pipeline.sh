set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr1
LANES=3 K=30 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1/p3 -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/tr1/p3.log 2>&1
LANES=1 K=20 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1/p1 -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/tr1/p1.log 2>&1
