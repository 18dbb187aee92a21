#!/bin/bash
# r06z: each resident wave's first item by its index (HRT_STATIC_FIRST A/B: a workgroup's 16 waves take 16
# neighbouring items of the longest-first plan, so its waves end together) -- the realtime loop, the batched
# launch, ranks 3 / 6 of 8, and the single-frame launch's workgroup hold (tools/wg_hold.py).
# builds: EXP_PATCH=tools/exp/r06yz_single_frame_threshold_static_first_rejected.patch bash tools/ab_build.sh sf1 -DHRT_STATIC_FIRST=1 (sftl: plus -DHRT_TIMELINE=1; rtf0: no definitions)
set -o pipefail
OUT=gpurun_out/r06z; mkdir -p $OUT
for r in 0 1; do
for v in rtf0 sf1; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 150 python3 tools/realtime.py --lanes 3 --busy-split 2 --rounds 1 ${SCENE_ARGS} > $OUT/rt_${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/rt_${v}_$r.jsonl; exit 1; }
  echo "== $v $r"; cat $OUT/rt_${v}_$r.jsonl
done
done
HRT_LIB=epq_raytracer_amd/build/ab_sftl/libhip_raytrace.so timeout -k 10 120 python3 tools/timeline.py --warmup 1 --steps 1 --raw $OUT/sf_single.npy --json $OUT/sf_single.json > $OUT/tl_sf_single.log 2>&1 || { echo "tl failed"; tail -5 $OUT/tl_sf_single.log; exit 1; }
python3 tools/wg_hold.py $OUT/sf_single.npy | tee $OUT/hold_sf_single.json || exit 1
for v in rtf0 sf1; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 200 python3 tools/rank_shape.py --rounds 2 --parts 3 6 > $OUT/rank_$v.jsonl 2>&1 || { echo "rank $v failed"; tail -3 $OUT/rank_$v.jsonl; exit 1; }
  echo "== rank $v"; grep -v summary $OUT/rank_$v.jsonl
done
