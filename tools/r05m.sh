#!/bin/bash
# r05m: whole-tile primary lists built once per launch by a tile_lists kernel (HRT_TL_PREPASS, in-tree =
# ab_prepass) against building them per item (ab_base): GPU suite (full), then rank_shape (whole frame +
# ranks 6, 2 of 8) x 3, cave whole + rank 6 x 2, and bench.py (ms per step, realtime loop) x 2.
set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for L in base prepass; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
  done
done
for r in 1 2; do
  for L in base prepass; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['per_frame_dispatch_ms'])" | tee -a $OUT/bench_ab.txt
  done
done
