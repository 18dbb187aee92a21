#!/bin/bash
# r03d: bounce-traversal diagnostics (pairs per bounce ray, band lengths) on cave and island, a cave
# bounce-batch sweep, and the A/B of the current library (per-scene band width) against HRT_WQ_TRI_MIN 32.
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
L=epq_raytracer_amd/build
timeout -k 10 300 python3 tools/kbench.py --variants 0 --rounds 2 --scene cave --diag --no-ref --sec-batch 0 24 48 64 > $OUT/diag_cave.jsonl 2>&1 || { echo "kbench cave failed"; tail -5 $OUT/diag_cave.jsonl; exit 1; }
timeout -k 10 300 python3 tools/kbench.py --variants 0 --rounds 1 --diag --no-ref > $OUT/diag_island.jsonl 2>&1 || { echo "kbench island failed"; tail -5 $OUT/diag_island.jsonl; exit 1; }
cat $OUT/diag_cave.jsonl $OUT/diag_island.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    if not l.startswith('{'): continue
    d = json.loads(l)
    if 'bvh_visits_per_lane' in d:
        print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items() if k in ('variant','bounce_lanes_per_iter','bvh_visits_per_lane','bvh_prims_per_lane','bvh_band_per_lane','bvh_trips_per_iter','band_len_per_lane','band_max_per_batch','bounce_cycle_share','primary_cycle_share','shade_cycle_share','bounce_iters','bounce_lanes')})
    elif 'ms_median' in d:
        print({k: d[k] for k in ('variant','sec_batch','ms_median','ms_min','mrays_s','lane_eff')})
"
LIBS="$L/ab_kargs2/libhip_raytrace.so $L/ab_cur/libhip_raytrace.so $L/ab_trimin32/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl $OUT/ab_island.jsonl
