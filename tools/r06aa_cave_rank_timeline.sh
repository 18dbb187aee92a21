#!/bin/bash
# r06aa: per-item timelines of cave's slowest rank of 8 (part 3) and a fast one (part 6) at bench.py's shape
# (5-frame warm-up, 20-frame timed launch; ab_timeline = -DHRT_TIMELINE=1 of HEAD)
set -o pipefail
OUT=gpurun_out/r06aa; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
for p in 3 6; do
timeout -k 10 150 python3 tools/timeline.py --scene cave --partition 8,$p,8 --raw $OUT/cave_rank$p.npy --json $OUT/cave_rank$p.json --costs $OUT/cave_rank${p}_costs.npy > $OUT/tl_cave_rank$p.log 2>&1 || { echo "rank$p failed"; tail -5 $OUT/tl_cave_rank$p.log; exit 1; }
done
echo done
