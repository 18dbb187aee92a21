#!/bin/bash
# r06ad: HRT_MULTI_FACTOR4 = 5 (mf5) against today's auto (mf0) at 8, 4 and 2 ranks, island and cave, bench.py's shape.
# builds: EXP_PATCH=tools/exp/r06ac_multi_factor_ab.patch bash tools/ab_build.sh mfN -DHRT_MULTI_FACTOR4=N (against the commit before the adopted change)
set -o pipefail
OUT=gpurun_out/r06ad; mkdir -p $OUT
for g in 8 4 2; do
for s in island cave; do
for v in mf0 mf5; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 280 python3 tools/rank_shape.py --gpus $g --scene $s --rounds 2 > $OUT/${s}_g${g}_$v.jsonl 2>&1 || { echo "$s $g $v failed"; tail -3 $OUT/${s}_g${g}_$v.jsonl; exit 1; }
  echo "== $s g$g $v"; tail -1 $OUT/${s}_g${g}_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['whole_kernel_ms'], [r['slowest_over_fair'] for r in d['runs']], [r['slowest_ms'] for r in d['runs']])"
done
done
done
