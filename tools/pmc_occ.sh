# Occupancy / stall counters of the 2^20 table-MSM kernels (one lane, serial).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
K=6 LANES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/occ/a -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/occ/a.log 2>&1
K=6 LANES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d gpurun_out/occ/b -o run -- python3 tools/perf_table.py 20 0:0 > gpurun_out/occ/b.log 2>&1
