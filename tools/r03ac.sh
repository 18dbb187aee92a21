#!/bin/bash
# r03ac: triangle-step threshold HRT_WQ_TRI_MIN 16 / 32 / 64 (current) / 128: ms per frame on island and
# cave, and the cave traversal counters (node / triangle pairs per bounce lane) of each build.
set -o pipefail
OUT=gpurun_out/r03ac; mkdir -p $OUT
L=epq_raytracer_amd/build
NAMES=${NAMES:-"cur tm16 tm32 tm128"}
LIBS=""; for B in $NAMES; do LIBS="$LIBS $L/ab_$B/libhip_raytrace.so"; done
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
for B in $NAMES; do
  HRT_LIB=$L/ab_$B/libhip_raytrace.so timeout -k 10 300 python3 tools/kbench.py --variants 0 --diag --scene cave --rounds 1 --no-ref > $OUT/diag_cave_$B.jsonl 2>&1 || { echo "diag $B failed"; tail -5 $OUT/diag_cave_$B.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$OUT/diag_cave_$B.jsonl'):
    if l.startswith('{') and 'bvh_band_per_lane' in l:
        d=json.loads(l); print('$B', {k: round(d[k],3) for k in ('bvh_visits_per_lane','bvh_prims_per_lane','bvh_band_per_lane','bvh_trips_per_iter','bounce_cycle_share')})
"
done
