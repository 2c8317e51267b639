set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py "tests/test_gpu_keygen.py::test_zbatch_full_keygen_prove_verify" > gpurun_out/r06a/tests.log 2>&1 && \
REPS=3 K=60 tools/env_ab.sh r06a/depth "d2|LANES=2 DEPTH=2" "d3|LANES=2 DEPTH=3" "d4|LANES=2 DEPTH=4" "l3d3|LANES=3 DEPTH=3"
