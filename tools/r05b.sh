#!/bin/bash
# r05b: (1) SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU on the exec-mask probe (lane-weighted VALU);
# (2) a rank of 8 at bench.py's shape: frames per launch 20 / 40 / 64 and the planner's split knobs
#     (ab_base = HEAD's kernel); (3) A/B: band offsets requested at the batch start (ab_bandearly).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r05b; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 -d $OUT/lanes -o run --output-format csv -- tools/probe/flops_probe > $OUT/lanes_probe.txt 2>&1 || { echo "lanes probe failed"; tail -5 $OUT/lanes_probe.txt; exit 1; }
export HRT_LIB=$B/ab_base/libhip_raytrace.so
for cfg in "--steps 20" "--steps 40" "--steps 64" "--option 5=16" "--option 5=64" "--option 6=1" "--option 6=4" "--option 7=0"; do
  timeout -k 10 120 python3 tools/rank_shape.py --rounds 2 --parts 6 $cfg > $OUT/rs.jsonl 2>&1 || { echo "rank shape $cfg failed"; tail -5 $OUT/rs.jsonl; exit 1; }
  echo "$cfg $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank6_knobs.txt
done
unset HRT_LIB
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_bandearly/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_bandearly/libhip_raytrace.so -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
