#!/bin/bash
# r04d: heavy items grabbed singly (sched[4] = the plan's heavy items), grab sizes for the light items,
# primary batching; parity subset first (split schedules, frame runs, multi-frame launches).
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "split_schedule or frame_runs or compute_n or sky or c5 or c4 or whole_frame or digest or bit_exact" -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
AB_BATCH=20 timeout -k 10 1000 bash tools/ab.sh 3 $L $B/ab_nolm/libhip_raytrace.so $B/ab_gh/libhip_raytrace.so $B/ab_g8/libhip_raytrace.so $B/ab_g6/libhip_raytrace.so $B/ab_pb8/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_nolm/libhip_raytrace.so $B/ab_gh/libhip_raytrace.so $B/ab_g8/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
# bounce-batch threshold re-sweep with the sky items out of the fused loop (HRT_OPT_SECONDARY_BATCH)
for r in 1 2; do for sb in 20 28 36 44 52; do
  out=$(timeout -k 10 120 python3 tools/frames.py --batch 20 --frames 3 --sec-batch $sb 2>&1 | tail -1) || { echo "sweep failed: $out"; exit 1; }
  echo "{\"round\": $r, \"sec_batch\": $sb, \"result\": $out}"
done; done > $OUT/sec_batch_island.jsonl
python3 -c "
import json,collections
b=collections.defaultdict(list)
for l in open('$OUT/sec_batch_island.jsonl'): d=json.loads(l); b[d['sec_batch']].append(min(d['result']['ms']))
print('sec_batch', {k: round(min(v),3) for k,v in b.items()})"
SKIP_TESTS=1 DIAG=1 bash tools/r04.sh r04d || exit 1
grep -h primary_iters $OUT/diag_island.jsonl $OUT/diag_cave.jsonl | python3 -c "import sys,json; [print('list entries tested: %.3f of %.2f per primary iteration' % (d['primary_survival'], d['primary_list_len'])) for d in map(json.loads, sys.stdin)]"
