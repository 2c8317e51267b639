#!/bin/bash
# round 6 A/B: headline loop and the bench's proof legs, baseline library
# (zelana_amd/_ab/libzkmi_base.so) against the tree's, interleaved.
set -o pipefail
OUT=gpurun_out/${TAG:-r06ab}
mkdir -p $OUT
cp zelana_amd/libzkmi.so zelana_amd/_ab/libzkmi_cur.so
for rep in 1 2 3; do
  for v in base cur; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=2 timeout -k 10 120 python3 tools/headline_loop.py 20 60 >> $OUT/ab.log 2>&1 || exit 1
  done
done
if [ -n "$LEGS" ]; then
  for rep in 1 2; do
    for v in base cur; do
      ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-plain --no-big \
        --no-window-ab --no-g2 --no-ntt --no-cpu-baseline $LEGS > $OUT/legs_${v}_$rep.json 2> $OUT/legs_${v}_$rep.err || exit 1
      python3 - $OUT/legs_${v}_$rep.json $v >> $OUT/ab.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
out = {"v": sys.argv[2], "head": d["value"]}
if "l2_proofs" in e:
    l = e["l2_proofs"]
    out.update(l2=l["proofs_per_s"], l2_two=l["two_in_flight"]["proofs_per_s"], matvec=l["stage_ms_per_proof"].get("g16_matvec"),
               pk_load=l.get("pk_load"))
if "zelana_batch_proofs" in e:
    z = e["zelana_batch_proofs"]
    out.update(zb=z["proofs_per_s"], zb_two=z["two_in_flight"]["proofs_per_s"], zb_pk_load=z.get("pk_load"))
if "config1_l2_small" in e:
    c = e["config1_l2_small"]
    out.update(c1_res=c["gpu_prove_resident_ms"], c1_nat=c["native_prove_ms"])
print(json.dumps(out))
PY
    done
  done
fi
cat $OUT/ab.log
