set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/brp2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm_ntt.py > gpurun_out/brp2/t.log 2>&1
LANES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/brp2/p -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/brp2/p.log 2>&1
LANES=2 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/brp2/p.log 2>&1
