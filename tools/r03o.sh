#!/bin/bash
# r03o: raygen without the sqrt / reciprocal of the second normalize (normalize_unit) and without the
# jitter's zero products: device math check, GPU suite, A/B timing against cur4.
set -o pipefail
OUT=gpurun_out/r03o; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -q -x -k "fast_division or camera_lists" --timeout 200 --timeout-method thread > $OUT/math.log 2>&1 || { echo "math check failed"; tail -30 $OUT/math.log; exit 1; }
tail -1 $OUT/math.log
timeout -k 10 600 bash tools/ab.sh 2 epq_raytracer_amd/build/ab_cur4/libhip_raytrace.so epq_raytracer_amd/lib/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 1 epq_raytracer_amd/build/ab_cur4/libhip_raytrace.so epq_raytracer_amd/lib/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl $OUT/ab_cave.jsonl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
