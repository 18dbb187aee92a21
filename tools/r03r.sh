#!/bin/bash
# r03r: runtime knob re-sweep after the r03 changes (bounce batch, leaf size, node-stack cap) on cave and
# island, and band cells of 512 per face edge (build A/B).
set -o pipefail
OUT=gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 900 bash tools/knobs.sh 2 cave "" "--sec-batch 20" "--sec-batch 36" "--sec-batch 44" "--leaf 2" "--leaf 4" "--ncap 512" > $OUT/knobs_cave.jsonl 2>&1 || { echo "cave knobs failed"; tail -3 $OUT/knobs_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/knobs_cave.jsonl
timeout -k 10 600 bash tools/knobs.sh 2 island "" "--sec-batch 24" "--sec-batch 32" "--leaf 3" > $OUT/knobs_island.jsonl 2>&1 || { echo "island knobs failed"; tail -3 $OUT/knobs_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/knobs_island.jsonl
L=epq_raytracer_amd
timeout -k 10 600 bash tools/ab.sh 2 $L/lib/libhip_raytrace.so $L/build/ab_dir512/libhip_raytrace.so -- --scene cave > $OUT/dir512_cave.jsonl 2>&1 || { echo "dir512 cave failed"; tail -3 $OUT/dir512_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/dir512_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $L/lib/libhip_raytrace.so $L/build/ab_dir512/libhip_raytrace.so > $OUT/dir512_island.jsonl 2>&1 || { echo "dir512 island failed"; tail -3 $OUT/dir512_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/dir512_island.jsonl
