#!/bin/bash
# NTT parity sizes + PMC issue figures of the 2^22 proof's accumulation kernels
set -o pipefail
OUT=gpurun_out/${TAG:-r06g2pmc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm_ntt.py -k ntt > $OUT/tests.log 2>&1 || { tail -n 20 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$OUT/pmc -o run -- python3 $R/tools/l2_loop.py 22 2 > $R/$OUT/pmc.log 2>&1 || exit 1
echo done
