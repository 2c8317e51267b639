set -e
mkdir -p gpurun_out/r03a
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a/tests.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
