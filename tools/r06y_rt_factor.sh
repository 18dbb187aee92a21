#!/bin/bash
# r06y: the realtime loop (3 lanes, busy split 2) with single-frame launches' heavy threshold at 0.5 / 1 / 1.5 x
# a wave's fair share (HRT_RT_FACTOR4 = 2 / 4 / 6 A/B builds) against today's 2 x (rtf0), island (SCENE_ARGS for others).
# builds: EXP_PATCH=tools/exp/r06yz_single_frame_threshold_static_first_rejected.patch bash tools/ab_build.sh rtfN -DHRT_RT_FACTOR4=N
set -o pipefail
OUT=gpurun_out/r06y; mkdir -p $OUT
for r in 0 1; do
for v in rtf0 rtf2 rtf4 rtf6; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 150 python3 tools/realtime.py --lanes 3 --busy-split 2 --rounds 1 ${SCENE_ARGS} > $OUT/${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/${v}_$r.jsonl; exit 1; }
  echo "== $v $r"; cat $OUT/${v}_$r.jsonl
done
done
