#!/bin/bash
# r04b: GPU suite + smoke, then A/B of frame runs, the handoff fences, the list-loop pairs, the sky
# loop's micro-variants (parity-checked first), and the sky / non-sky split timing (timing-only builds,
# tools/exp/r04_sky_split_timing.patch).
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
[ -z "$SKIP_SUITE" ] && { DIAG=1 bash tools/r04.sh r04b || exit 1; }
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
HRT_LIB=$B/ab_skyzn/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "sky or frame_bit_exact or split_schedule" -q -x --timeout 200 --timeout-method thread > $OUT/skyzn_parity.log 2>&1 || { echo "skyzn parity failed"; tail -30 $OUT/skyzn_parity.log; exit 1; }
tail -1 $OUT/skyzn_parity.log
AB_BATCH=20 timeout -k 10 1100 bash tools/ab.sh 2 $L $B/ab_norun/libhip_raytrace.so $B/ab_nofence/libhip_raytrace.so $B/ab_pairs/libhip_raytrace.so $B/ab_early/libhip_raytrace.so $B/ab_pb8/libhip_raytrace.so $B/ab_skyzn/libhip_raytrace.so $B/ab_grab8/libhip_raytrace.so $B/ab_dual32/libhip_raytrace.so $B/ab_nonsky/libhip_raytrace.so $B/ab_skyonly/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_norun/libhip_raytrace.so $B/ab_dual32/libhip_raytrace.so $B/ab_dual64/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
