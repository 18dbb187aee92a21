#!/bin/bash
# r05w: per-cell band records (a bounce lane's cell start + length + first 12 entries in one 32 B record;
# in-tree = ab_rec) against the 1024-cell lists with offsets (ab_prev): full GPU suite on the product,
# then whole frame + rank 6 (rank_shape) for island x3 and cave x2, interleaved.
set -o pipefail
OUT=gpurun_out/r05w; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for r in 1 2 3; do
  for S in island cave; do
    [ $S = cave ] && [ $r = 3 ] && continue
    for L in prev rec; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
