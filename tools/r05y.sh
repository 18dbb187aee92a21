#!/bin/bash
# r05y: the tile pixel pool in frame runs (HRT_PIXEL_POOL, in-tree = ab_pool) against per-lane runs
# (ab_nopool = the r05v kernel): full GPU suite on the product, then bench.py x2 (island + cave) and
# whole frame + rank 6 (rank_shape) x2.
set -o pipefail
OUT=gpurun_out/r05y; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for r in 1 2; do
  for L in nopool pool; do
    LIB=$B/ab_$L/libhip_raytrace.so
    HRT_LIB=$LIB timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L island bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['per_frame_dispatch_ms'])" | tee -a $OUT/bench_ab.txt
    HRT_LIB=$LIB timeout -k 10 300 python3 bench.py --scene cave --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench cave $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L cave bench', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/bench_ab.txt
  done
done
for r in 1 2; do
  for S in island cave; do
    for L in nopool pool; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
