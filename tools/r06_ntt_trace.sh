#!/bin/bash
# per-pass NTT kernel durations and HBM counters (2^24 NTT+INTT loop)
set -o pipefail
OUT=gpurun_out/${TAG:-r06ntt_tr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/tr -o run -- python3 $R/tools/ntt_loop.py 24 6 > $R/$OUT/tr.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$OUT/pmc1 -o run -- python3 $R/tools/ntt_loop.py 24 6 > $R/$OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$OUT/pmc2 -o run -- python3 $R/tools/ntt_loop.py 24 6 > $R/$OUT/pmc2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/$OUT/pmc3 -o run -- python3 $R/tools/ntt_loop.py 24 6 > $R/$OUT/pmc3.log 2>&1 || exit 1
find $R/$OUT -name "*.csv" | head -20
