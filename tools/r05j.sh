#!/bin/bash
# r05j: two-ended work queue (one wave per SIMD takes the cheapest items from the far end), the tile-list
# prefetch and the sky d.y-only normalize.  GPU suite subset on the in-tree build (all three), then
# bench-shape rank_shape (whole + ranks 6, 2 of 8) for ab_base / ab_te_only / ab_twoend (all three), and the
# frames.py A/B (20-frame launches) of the two small changes alone against ab_base.
set -o pipefail
OUT=gpurun_out/r05j; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for L in base te_only twoend; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
  done
done
for r in 1 2; do
  for L in base te_only; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_prefetch/libhip_raytrace.so $B/ab_skydy/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
