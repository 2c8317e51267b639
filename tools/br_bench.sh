# Bench legs (2^20 headline, L2 2^22 proofs, zelana_batch) with the round-1
# bucket reduction (ZKMI_BR_MODE=1) and the fold + lines form (default).
set -e
mkdir -p gpurun_out/brb
for rep in 1 2; do
for m in 1 2; do
  ZKMI_BR_MODE=$m timeout -k 10 300 python3 bench.py --steps 30 --no-cpu-baseline --no-big --no-plain --no-ntt > gpurun_out/brb/m$m.$rep.json 2> gpurun_out/brb/m$m.$rep.err
done
done
