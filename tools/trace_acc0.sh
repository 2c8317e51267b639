set -e
for t in 768 1024 4096; do ZKMI_LIB=zelana_amd/variants/libzkmi_trace.so ZKMI_ACC_TPC=$t timeout -k 10 120 python3 tools/trace_acc0.py; done
