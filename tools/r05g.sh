#!/bin/bash
# r05g: frame runs on ranks of 8 -- the singly grabbed tail capped at 1/4 or 1/2 of the launch's items
# (HRT_TAIL_DIV), long tiles (>= a wave's launch work / 8) singly, at priority (div4, div2) or not (div4c),
# against ab_base and lhot8; rank_shape, 3 rounds each, ranks 6 and 2 of 8 + the whole frame.
set -o pipefail
OUT=gpurun_out/r05g; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2 3; do
  for L in base lhot8 div4 div2 div4c; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
  done
done
