#!/bin/bash
# r06u: the warm-up launch's per-tile costs (hrt_debug_tile_costs) beside the timed launch's per-item timeline
# (ab_timeline), rank 3 of 8 with 5 and 40 warm-up frames, and the whole frame.
set -o pipefail
OUT=gpurun_out/r06u; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
for w in 5 40; do
timeout -k 10 150 python3 tools/timeline.py --partition 8,3,8 --warmup $w --raw $OUT/rank3_w$w.npy --costs $OUT/rank3_w${w}_costs.npy --json $OUT/rank3_w$w.json > $OUT/tl_rank3_w$w.log 2>&1 || { echo "rank3 w$w failed"; tail -5 $OUT/tl_rank3_w$w.log; exit 1; }
done
timeout -k 10 150 python3 tools/timeline.py --warmup 5 --raw $OUT/whole_w5.npy --costs $OUT/whole_w5_costs.npy --json $OUT/whole_w5.json > $OUT/tl_whole.log 2>&1 || { echo "whole failed"; tail -5 $OUT/tl_whole.log; exit 1; }
ls $OUT
