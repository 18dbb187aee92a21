#!/bin/bash
# r05o: mutation check -- a build whose tile-list key is the camera position only and which keeps the lists
# across hrt_generate_rays (tools/exp/r05_tile_list_key_mutant.patch) must fail the tile-list test, and the
# product build pass it.
set -o pipefail
OUT=gpurun_out/r05o; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -q -x -k "tile_lists or camera_lists" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "product tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
if HRT_LIB=$B/ab_mutant/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -q -k "tile_lists" --timeout 200 --timeout-method thread > $OUT/mutant_tests.log 2>&1; then
  echo "MUTANT SURVIVED"; tail -3 $OUT/mutant_tests.log
else
  echo "mutant caught:"; grep -E "^E .*(frame|regenerated)" $OUT/mutant_tests.log | head -4; tail -1 $OUT/mutant_tests.log
fi
