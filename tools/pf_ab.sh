# Sort-scatter prefetch A/B: in-tree build (ZK_RS_PF=1) vs zelana_amd/_ab/libzkmi_pf0.so.
set -e
mkdir -p gpurun_out/pf
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm_ntt.py > gpurun_out/pf/t.log 2>&1
for rep in 1 2; do
for v in pf1 pf0; do
  if [ $v = pf0 ]; then export ZKMI_LIB=zelana_amd/_ab/libzkmi_pf0.so; else unset ZKMI_LIB; fi
  echo "== 20 $v" >> gpurun_out/pf/p.log
  LANES=1,3 timeout -k 10 120 python3 tools/perf_table.py 20 0:0 >> gpurun_out/pf/p.log 2>&1
  echo "== 26 $v" >> gpurun_out/pf/p.log
  K=6 LANES=1,2 timeout -k 10 200 python3 tools/perf_table.py 26 0:0 >> gpurun_out/pf/p.log 2>&1
done
done
