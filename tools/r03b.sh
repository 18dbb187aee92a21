#!/bin/bash
# r03b: realtime deferred-combine A/B, cave phase costs (HRT_EXP_TWICE builds), PMC records of the current build.
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT
L=epq_raytracer_amd
timeout -k 10 300 python3 tools/realtime.py --lanes 3 --busy-split 1 2 --defer 0 1 --rounds 2 > $OUT/realtime.jsonl 2>&1 || { echo "realtime failed"; tail -5 $OUT/realtime.jsonl; exit 1; }
cat $OUT/realtime.jsonl
timeout -k 10 600 bash tools/ab.sh 3 $L/build/ab_base/libhip_raytrace.so $L/build/ab_kargs/libhip_raytrace.so $L/build/ab_kargs2/libhip_raytrace.so $L/build/ab_lean/libhip_raytrace.so > $OUT/kargs_island.jsonl 2>&1 || { echo "ab kargs failed"; tail -5 $OUT/kargs_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $L/build/ab_base/libhip_raytrace.so $L/build/ab_kargs/libhip_raytrace.so $L/build/ab_kargs2/libhip_raytrace.so $L/build/ab_lean/libhip_raytrace.so -- --scene cave > $OUT/kargs_cave.jsonl 2>&1 || { echo "ab kargs cave failed"; tail -5 $OUT/kargs_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/kargs_island.jsonl $OUT/kargs_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $L/lib/libhip_raytrace.so $L/build/ab_exp1/libhip_raytrace.so $L/build/ab_exp2/libhip_raytrace.so $L/build/ab_exp3/libhip_raytrace.so $L/build/ab_exp5/libhip_raytrace.so -- --scene cave > $OUT/phase_cave.jsonl 2>&1 || { echo "ab failed"; tail -5 $OUT/phase_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/phase_cave.jsonl
bash tools/pmc.sh r03b/pmc_cave --scene cave > $OUT/pmc_cave.log 2>&1 || { echo "pmc cave failed"; tail -20 $OUT/pmc_cave.log; exit 1; }
bash tools/pmc.sh r03b/pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
python3 -c "
import json
for t in ('pmc', 'pmc_cave'):
    d = json.load(open('$OUT/%s/pmc_traffic.json' % t)); c = d['counters_per_launch']; f = d['frames_per_launch']
    print(t, d['kernel'], 'frames', f, 'ms/frame', round(d['launch_duration_s'] / f * 1e3, 3), 'VALU/frame G', round(c['SQ_INSTS_VALU'] / f / 1e9, 3),
          'SALU/VALU', round(c['SQ_INSTS_SALU'] / c['SQ_INSTS_VALU'], 3), 'LDS/frame G', round(c['SQ_INSTS_LDS'] / f / 1e9, 3),
          'FP32 TF', round(d['executed_fp32_tflops'], 2), 'HBM GB/frame', round(d['hbm_bytes_per_frame'] / 1e9, 3), 'wait', round(d['wait_any_frac'], 3), 'valu_util', round(d['valu_issue_utilisation'], 3))
"
