#!/bin/bash
# r06k: the heavy-tile threshold at 1/2, 1/4, 1/8 of a wave's fair share (HRT_HEAVY_DIV A/B builds): ranks 3 and 6
# of 8 and the whole frame at bench.py's shape (tools/rank_shape.py), island.
set -o pipefail
OUT=gpurun_out/r06k; mkdir -p $OUT
for v in base hdiv2 hdiv4 hdiv8; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == base ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --rounds 1 --parts 3 6 ${SCENE_ARGS} > $OUT/$v.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.jsonl; exit 1; }
  echo "== $v"; grep -v summary $OUT/$v.jsonl
done
