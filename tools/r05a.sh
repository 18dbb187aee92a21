#!/bin/bash
# r05a: (1) does SQ_INSTS_VALU_FLOPS_FP32 weight by the exec mask (tools/probe/flops_probe.hip);
# (2) BUNDLE_WQ node-step fill and member-slot use on island and cave (HRT_DIAG_WQ_*, the r04 step: ab_base);
# (3) the spread node step (HRT_WQ_SPREAD, in-tree build): GPU suite subset, then timing against ab_base.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r05a; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 -d $OUT/flops -o run --output-format csv -- tools/probe/flops_probe > $OUT/flops_probe.txt 2>&1 || { echo "flops probe failed"; tail -5 $OUT/flops_probe.txt; exit 1; }
grep '^{' $OUT/flops_probe.txt
HRT_LIB=$B/ab_base/libhip_raytrace.so timeout -k 10 300 python3 tools/kbench.py --variants 9 --rounds 1 --no-ref --diag > $OUT/diag_island.jsonl 2>&1 || { echo "diag island failed"; tail -5 $OUT/diag_island.jsonl; exit 1; }
HRT_LIB=$B/ab_base/libhip_raytrace.so timeout -k 10 300 python3 tools/kbench.py --variants 9 --rounds 1 --no-ref --diag --scene cave > $OUT/diag_cave.jsonl 2>&1 || { echo "diag cave failed"; tail -5 $OUT/diag_cave.jsonl; exit 1; }
grep -h '"wq_' $OUT/diag_*.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k: round(v,4) if isinstance(v,float) else v for k,v in d.items() if k.startswith('wq_') or k in ('bvh_visits_per_lane','bvh_trips_per_iter','bounce_lanes_per_iter')})"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_spread/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_spread/libhip_raytrace.so -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
HRT_LIB=$B/ab_base/libhip_raytrace.so timeout -k 10 300 python3 tools/rank_shape.py --rounds 2 > $OUT/rank8_base.jsonl 2>&1 || { echo "rank shape failed"; tail -5 $OUT/rank8_base.jsonl; exit 1; }
tail -1 $OUT/rank8_base.jsonl
