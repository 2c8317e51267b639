set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trlv
for v in cur w2; do
ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=1 K=10 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trlv/$v.1 -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/trlv/$v.1.log 2>&1
ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=3 K=20 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trlv/$v.3 -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/trlv/$v.3.log 2>&1
done
