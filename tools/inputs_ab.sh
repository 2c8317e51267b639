# Headline MSM with the §8d StdRng input streams vs the round-1 splitmix streams.
set -e
mkdir -p gpurun_out/inab
for rep in 1 2; do
for k in stdrng splitmix; do
  timeout -k 10 200 python3 bench.py --inputs $k --no-l2 --no-zbatch --no-ntt --no-plain --no-big --no-cpu-baseline --steps 40 > gpurun_out/inab/$k.$rep.json 2>/dev/null
done
done
