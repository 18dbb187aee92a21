#!/bin/bash
# r06w: plan costs as an exponential average over a lane's launches (HRT_COST_DECAY 1 / 2 A/B builds) against
# the product (costs of the last launch only): the realtime loop (tools/realtime.py, 3 lanes, busy split 2),
# then ranks 3 and 6 of 8 and the whole frame at bench.py's shape.
set -o pipefail
OUT=gpurun_out/r06w; mkdir -p $OUT
for r in 1 2; do
for v in base decay1 decay2; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == base ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/realtime.py --lanes 3 --busy-split 2 --defer 0 --rounds 1 > $OUT/rt_${v}_$r.jsonl 2>&1 || { echo "$v rt failed"; tail -3 $OUT/rt_${v}_$r.jsonl; exit 1; }
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --rounds 1 --parts 3 6 > $OUT/rank_${v}_$r.jsonl 2>&1 || { echo "$v rank failed"; tail -3 $OUT/rank_${v}_$r.jsonl; exit 1; }
  echo "== $v $r realtime $(python3 -c "import json; print([json.loads(l)['ms_per_frame'] for l in open('$OUT/rt_${v}_$r.jsonl') if l.startswith('{')])") ranks $(grep -v summary $OUT/rank_${v}_$r.jsonl | python3 -c 'import sys,json; print([json.loads(l)["kernel_ms"] for l in sys.stdin])')"
done; done
