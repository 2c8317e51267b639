# L2 prove at 2^22 with the default table windows and with pk tables pinned to c=17
set -e
timeout -k 10 300 python3 tools/perf_l2.py 22 > gpurun_out/l2_auto.log 2>&1
ZKMI_TABLE_C=17 timeout -k 10 300 python3 tools/perf_l2.py 22 > gpurun_out/l2_c17.log 2>&1
