#!/bin/bash
# r05ab: frame runs in short planned launches (HRT_RUN_SHORT: tiles <= 1/HRT_RUN_SHORT_DIV of a wave's
# share grabbed 4 at a time, last HRT_RUN_SHORT_TAIL items per wave singly): base (off), rs64, rs32,
# rs128, rs64t8 -- GPU suite on the product, then whole frame + ranks 6 and 3 of 8, island and cave x2.
set -o pipefail
OUT=gpurun_out/r05ab; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for r in 1 2; do
  for S in island cave; do
    for L in base rs64 rs32 rs128 rs64t8; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 3 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
