# Dev sweep (GPU box): headline 2^20 table MSM under env knobs, 3 lanes.
set -e
mkdir -p gpurun_out/sk
F="--no-plain --no-ntt --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 40"
run() {  # name env...
  n=$1; shift
  env "$@" timeout -k 10 120 python bench.py $F > gpurun_out/sk/$n.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/sk/$n.json'));print('$n', d['value'], d['ms_per_step'], d['extra']['msm_stage_ms_per_step'])"
}
run base ZKMI_X=0
run strip4 ZKMI_BR_STRIP=4
run strip16 ZKMI_BR_STRIP=16
run c19 ZKMI_TABLE_C=19
run c21 ZKMI_TABLE_C=21
run st1_2048 ZKMI_RS_ST1=2048
run st1_8192 ZKMI_RS_ST1=8192
run base2 ZKMI_X=0
