#!/bin/bash
# round 6 A/B over zelana_amd/_ab/libzkmi_<v>.so variants (VARIANTS), interleaved:
# the 2^22 proof loop (tools/l2_loop.py, one and two in flight) and, with LEGS,
# bench.py's proof legs (headline + config-4/zelana_batch/config-1)
set -o pipefail
OUT=gpurun_out/${TAG:-r06ab2}
mkdir -p $OUT
for v in ${VTEST:-}; do
  ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu ${TESTS:-tests/test_gpu_groth16.py} > $OUT/tests_$v.log 2>&1 || { tail -n 20 $OUT/tests_$v.log; exit 1; }
  tail -n 1 $OUT/tests_$v.log
done
for rep in 1 2; do
  for v in ${VARIANTS:-base}; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 200 python3 tools/l2_loop.py 22 10 >> $OUT/ab.log 2>&1 || exit 1
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so TWO=1 timeout -k 10 200 python3 tools/l2_loop.py 22 10 >> $OUT/ab.log 2>&1 || exit 1
    if [ -n "$LEGS" ]; then
      ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-plain --no-big \
        --no-window-ab --no-g2 --no-ntt --no-cpu-baseline --no-l2 > $OUT/legs_${v}_$rep.json 2> $OUT/legs_${v}_$rep.err || exit 1
      python3 - $OUT/legs_${v}_$rep.json $v >> $OUT/ab.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
z, c = e["zelana_batch_proofs"], e.get("config1_l2_small", {})
print(json.dumps({"v": sys.argv[2], "zb": z["proofs_per_s"], "zb_two": z["two_in_flight"]["proofs_per_s"],
                  "zb_e2e4": z["end_to_end"]["batched"]["proofs_per_s"], "c1_res": c.get("gpu_prove_resident_ms"),
                  "c1_nat": c.get("native_prove_ms")}))
PY
    fi
  done
done
cat $OUT/ab.log
