#!/bin/bash
# r05e: long tiles singly + frame runs for the rest (HRT_LONG_L 8) with grab tails of 64 / 16 / 8 items per
# wave, against the r04 rule (ab_base), at bench.py's shape: the whole frame and ranks 6 and 2 of 8; then
# cave's whole frame.
set -o pipefail
OUT=gpurun_out/r05e; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2; do
  for L in base long_t64 long_t16 long_t8; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
