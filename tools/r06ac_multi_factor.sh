#!/bin/bash
# r06ac: many-frame launches' heavy threshold at 1 / 1.25 / 1.5 x a wave's share of the launch (HRT_MULTI_FACTOR4
# = 4 / 5 / 6 A/B builds; mf0 = today's auto, 2 x at these shapes) -- ranks of 8 at bench.py's shape, cave and island.
set -o pipefail
# builds: EXP_PATCH=tools/exp/r06ac_multi_factor_ab.patch bash tools/ab_build.sh mfN -DHRT_MULTI_FACTOR4=N (against the commit before the adopted change)
OUT=gpurun_out/r06ac; mkdir -p $OUT
for s in cave island; do
for v in mf0 mf4 mf5 mf6; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 280 python3 tools/rank_shape.py --scene $s --rounds 2 > $OUT/${s}_$v.jsonl 2>&1 || { echo "$s $v failed"; tail -3 $OUT/${s}_$v.jsonl; exit 1; }
  echo "== $s $v"; tail -1 $OUT/${s}_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['whole_kernel_ms'], [r['slowest_over_fair'] for r in d['runs']], {k: v for k, v in d['part_kernel_ms'].items()})"
done
done
