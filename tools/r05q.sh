#!/bin/bash
# r05q: grazing-band direction cells per cube-face edge for small scenes (HRT_DIR_RES_SMALL 256 = ab_base,
# 384, 512): whole frame + rank 6 of 8 at bench.py's shape, island x3 and cave x2, interleaved.
set -o pipefail
OUT=gpurun_out/r05q; mkdir -p $OUT
B=epq_raytracer_amd/build
for L in dr384 dr512; do
  HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "headline or golden or grazing or wq_node_radius or frame_bit_exact or degenerate" --timeout 300 --timeout-method thread > $OUT/tests_$L.log 2>&1 || { echo "tests $L failed"; tail -30 $OUT/tests_$L.log; exit 1; }
  echo "$L $(tail -1 $OUT/tests_$L.log)"
done
for r in 1 2 3; do
  for L in base dr384 dr512; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
  done
done
for r in 1 2; do
  for L in base dr384 dr512; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
