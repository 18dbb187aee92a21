#!/bin/bash
# r04w: shading takes the draws after the invisible-object test (is_spec's hash, the diffuse unit-sphere
# draw) on a copy of the RNG state while the material and normal loads are in flight, committing the
# state where the path goes on.  Parity subset on the in-tree build, then timing against the r04t
# build (ab_cone2).
set -o pipefail
OUT=gpurun_out/r04w; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $B/ab_cone2/libhip_raytrace.so $B/ab_spec/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_cone2/libhip_raytrace.so $B/ab_spec/libhip_raytrace.so -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
