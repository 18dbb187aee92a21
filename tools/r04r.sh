#!/bin/bash
# r04r: sky-loop trims (normalize_wu's fast flag: no 1.5 checks, no 0 + light; ballots of the compares;
# u01 scalings folded) and the per-wave normalize in the fused loop (HRT_NORM_UNIFORM_FUSED=1, ab_skyfu).
# Parity of ab_skyfu first (both changes), then interleaved timing against the r04l build (ab_base).
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
B=epq_raytracer_amd/build
HRT_LIB=$B/ab_skyfu/libhip_raytrace.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_sky/libhip_raytrace.so $B/ab_skyfu/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_sky/libhip_raytrace.so $B/ab_skyfu/libhip_raytrace.so -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
