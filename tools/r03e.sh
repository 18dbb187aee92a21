#!/bin/bash
# r03e: per-triangle node margins (pertri) and the margin-aware SAH (sahr10 / sahr25) against the current
# library on cave and island; cave bounce-batch sweep (compute_n, 64-frame launches).
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_pertri/libhip_raytrace.so $L/ab_sahr10/libhip_raytrace.so $L/ab_sahr25/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl $OUT/ab_island.jsonl
for sb in 28 36 48 64; do
  HRT_LIB=$L/ab_pertri/libhip_raytrace.so timeout -k 10 120 python3 tools/frames.py --scene cave --batch 64 --frames 2 --sec-batch $sb 2>&1 | tail -1
done > $OUT/secbatch_cave.jsonl || { echo "sec batch sweep failed"; exit 1; }
cat $OUT/secbatch_cave.jsonl
