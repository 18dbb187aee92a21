#!/bin/bash
# r05f: long tiles (cost >= a wave's launch work / L, L = 4 / 8 / 16) grabbed singly AND at the heavy tiles'
# issue priority (HRT_LONG_HOT), against ab_base (r04 rule) and ab_long_t64 (long, no priority), at
# bench.py's shape: the whole frame and ranks 6 and 2 of 8 (island), rank 6 of 8 (cave).
set -o pipefail
OUT=gpurun_out/r05f; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2; do
  for L in base long_t64 lhot4 lhot8 lhot16; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
