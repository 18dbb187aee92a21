#!/bin/bash
# r05h: the small-launch plan (in-tree build = ab_small): GPU suite subset, then rank_shape against ab_base
# (3 rounds: whole frame + ranks 6 and 2 of 8, island; whole + rank 6, cave), then all 8 ranks of island.
set -o pipefail
OUT=gpurun_out/r05h; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for L in base small; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
timeout -k 10 300 python3 tools/rank_shape.py --rounds 2 > $OUT/rank8_small.jsonl 2>&1 || { echo "rank8 failed"; tail -5 $OUT/rank8_small.jsonl; exit 1; }
tail -1 $OUT/rank8_small.jsonl
