#!/bin/bash
# r03v: band-flatten owner fix (relaxed LDS atomics for the start marks) -- the new debug check against the
# fixed library and against a build with the old plain accesses (expected to fail); A/B of branch-free
# member / band pushes (dump); the whole GPU suite on the production library.
set -o pipefail
OUT=gpurun_out/r03v; mkdir -p $OUT
L=epq_raytracer_amd/build
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -m gpu -q -k band_flatten --timeout 120 --timeout-method thread > $OUT/flatten_fixed.log 2>&1 || { echo "flatten test failed on the fixed library"; tail -30 $OUT/flatten_fixed.log; exit 1; }
tail -1 $OUT/flatten_fixed.log
HRT_LIB=$L/ab_bandbug/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -m gpu -q -k band_flatten --timeout 120 --timeout-method thread > $OUT/flatten_oldbuild.log 2>&1
echo "old-build flatten rc=$? (expected non-zero)"; grep -E "passed|failed" $OUT/flatten_oldbuild.log | tail -1
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_dump/libhip_raytrace.so $L/ab_bandbug/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
