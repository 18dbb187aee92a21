#!/bin/bash
# r05ag: the tile-list prepass (HRT_TL_PREPASS) on the final kernel: product (ab_pbase) against no prepass
# (ab_notl), whole frame + rank 6, island and cave x3.
set -o pipefail
OUT=gpurun_out/r05ag; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2 3; do
  for S in island cave; do
    for L in pbase notl; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
