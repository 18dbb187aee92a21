#!/bin/bash
# r05ah: band width tau_g 4e-3 (ab_t4) against 3e-3 (ab_pbase) on the final kernel: whole frame + ranks
# 6 and 3 of 8 at bench.py's shape, island and cave x3.
set -o pipefail
OUT=gpurun_out/r05ah; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2 3; do
  for S in island cave; do
    for L in pbase t4; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 3 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
