set -e
mkdir -p gpurun_out/sw
F="--no-plain --no-ntt --no-l2 --no-zbatch --no-big --no-cpu-baseline --steps 40"
for l in 3 4 5 3 4 5; do
  timeout -k 10 120 python bench.py $F --lanes $l > gpurun_out/sw/l$l.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/sw/l$l.json'));print('lanes $l', d['value'], d['ms_per_step'])"
done
