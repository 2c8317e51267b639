set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
for rep in 1 2 3; do
  for v in base loose; do
    echo "== $v rep $rep" >> $OUT/ab.log
    ZKMI_LIB=zelana_amd/_ab/libzkmi_$v.so LANES=2 DEPTH=2 timeout -k 10 120 python3 tools/headline_loop.py 20 60 >> $OUT/ab.log 2>&1 || exit 1
  done
done
cat $OUT/ab.log
