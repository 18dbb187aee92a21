#!/bin/bash
# r05ae: three kernel switches re-checked on the final kernel (1024 band cells, pixel pool): the bounce
# lane's band offsets requested at the batch's start (HRT_WQ_BAND_EARLY=1), no bounce issue priority
# (HRT_BOUNCE_PRIO=0), two sky samples per trip (HRT_SKY_UNROLL=2); whole frame + rank 6, island and cave x2.
set -o pipefail
OUT=gpurun_out/r05ae; mkdir -p $OUT
B=epq_raytracer_amd/build
HRT_LIB=$B/ab_early/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "headline or golden or grazing or wq_node_radius or frame_runs" --timeout 200 --timeout-method thread > $OUT/tests_early.log 2>&1 || { echo "tests early failed"; tail -30 $OUT/tests_early.log; exit 1; }
echo "early $(tail -1 $OUT/tests_early.log)"
for r in 1 2; do
  for S in island cave; do
    for L in pbase early prio0 sky2; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
