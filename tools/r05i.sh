#!/bin/bash
# r05i: cost-capped frame runs + guided grabs (HRT_GUIDED, in-tree = ab_guided; run budget 1/8 of a wave's
# launch work, grabs <= remaining / (2 x resident)) and variants (budget 1/4, 1/16; remaining / 4R) against
# the r04 grabs (ab_base): GPU suite subset first, then rank_shape (whole frame + ranks 6, 2 of 8) x 3.
set -o pipefail
OUT=gpurun_out/r05i; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for L in base guided g_b4 g_b16 g_c4; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 2 > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_island.txt
  done
done
for r in 1 2; do
  for L in base guided g_b4 g_b16; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene cave > $OUT/rs.jsonl 2>&1 || { echo "cave rank shape $L failed"; tail -5 $OUT/rs.jsonl; exit 1; }
    echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_cave.txt
  done
done
timeout -k 10 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1; grep -i -B2 -A8 "pc.sampl\|PC_SAMPL" $OUT/list_avail.txt | head -40
# sky segment: d.y-only second normalize (ab_skydy) against the same build without it (ab_base2)
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base2/libhip_raytrace.so $B/ab_skydy/libhip_raytrace.so > $OUT/ab_skydy_island.jsonl 2>&1 || { echo "ab skydy failed"; tail -5 $OUT/ab_skydy_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_skydy_island.jsonl
