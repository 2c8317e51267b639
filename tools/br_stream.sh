# Decoupled bucket reduction (shared br stream): correctness, then the
# pipelined 2^20 table MSM at 2-3 lanes with 2..5 MSMs in flight.
set -e
mkdir -p gpurun_out/brs
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py tests/test_gpu_groth16.py > gpurun_out/brs/t.log 2>&1
for rep in 1 2; do
for cfg in "LANES=3 DEPTH=3" "LANES=3 DEPTH=4" "LANES=3 DEPTH=5" "LANES=2 DEPTH=2" "LANES=2 DEPTH=3" "LANES=2 DEPTH=4"; do
  echo "== $cfg" >> gpurun_out/brs/p.log
  env $cfg timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/brs/p.log 2>&1
done
done
