#!/bin/bash
# r06x: per-item timelines of single-frame launches (the realtime loop's shape) -- how long each workgroup
# holds its CU past its waves' work (tools/wg_hold.py).
set -o pipefail
OUT=gpurun_out/r06x; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
for w in 1 5; do
timeout -k 10 120 python3 tools/timeline.py --warmup $w --steps 1 --raw $OUT/single_w$w.npy --json $OUT/single_w$w.json > $OUT/tl_single_w$w.log 2>&1 || { echo "single w$w failed"; tail -5 $OUT/tl_single_w$w.log; exit 1; }
python3 tools/wg_hold.py $OUT/single_w$w.npy > $OUT/hold_single_w$w.json || exit 1
done
timeout -k 10 120 python3 tools/timeline.py --scene cave --warmup 1 --steps 1 --raw $OUT/cave_single.npy --json $OUT/cave_single.json > $OUT/tl_cave_single.log 2>&1 || { echo "cave failed"; tail -5 $OUT/tl_cave_single.log; exit 1; }
python3 tools/wg_hold.py $OUT/cave_single.npy > $OUT/hold_cave_single.json || exit 1
cat $OUT/hold_*.json
