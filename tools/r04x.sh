#!/bin/bash
# r04x: a node step skipping its second member pair when no group in it has a third member
# (HRT_WQ_SKIP_PAIR2, in-tree), and the triangle-step threshold at 32 / 128 pairs (ab_tri32, ab_tri128;
# r04t build = ab_cone2, threshold 64).  Parity subset on the in-tree build first.
set -o pipefail
OUT=gpurun_out/r04x; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L="$B/ab_cone2/libhip_raytrace.so $B/ab_skip2/libhip_raytrace.so $B/ab_tri32/libhip_raytrace.so $B/ab_tri128/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
