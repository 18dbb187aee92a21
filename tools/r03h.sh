#!/bin/bash
# r03h: primary-list prefetch A/B (island, cave), island phase costs (HRT_EXP_TWICE builds), and a
# kernel trace of the realtime loop (trace/accumulate per frame) to see where per-frame dispatch loses
# time against hrt_compute_n.
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
L=epq_raytracer_amd/build
timeout -k 10 600 bash tools/ab.sh 2 $L/ab_cur3/libhip_raytrace.so $L/ab_prefetch/libhip_raytrace.so > $OUT/prefetch_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/prefetch_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $L/ab_cur3/libhip_raytrace.so $L/ab_prefetch/libhip_raytrace.so -- --scene cave > $OUT/prefetch_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/prefetch_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/prefetch_island.jsonl $OUT/prefetch_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $L/ab_cur3/libhip_raytrace.so $L/ab_exp1/libhip_raytrace.so $L/ab_exp2/libhip_raytrace.so $L/ab_exp3/libhip_raytrace.so $L/ab_exp4/libhip_raytrace.so $L/ab_exp5/libhip_raytrace.so > $OUT/phase_island.jsonl 2>&1 || { echo "ab phases failed"; tail -5 $OUT/phase_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/phase_island.jsonl
HRT_LIB=$L/ab_cur3/libhip_raytrace.so timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/rt -o run --output-format csv -- python3 tools/realtime.py --lanes 1 3 --busy-split 1 2 --defer 0 --rounds 1 --frames 24 > $OUT/realtime.log 2>&1 || { echo "realtime trace failed"; tail -20 $OUT/realtime.log; exit 1; }
grep ms_per_frame $OUT/realtime.log
echo done
