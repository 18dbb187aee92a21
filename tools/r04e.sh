#!/bin/bash
# r04e: realtime-loop knobs (trace lanes, busy split, deferred combines) and the planner's split knobs
# re-swept with the sky items and frame runs (island and cave, 20-frame launches).
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 300 python3 tools/realtime.py --lanes 2 3 --busy-split 1 2 3 4 --defer 0 1 --rounds 2 > $OUT/realtime.jsonl 2>&1 || { echo "realtime failed"; tail -5 $OUT/realtime.jsonl; exit 1; }
python3 -c "
import json,collections
b=collections.defaultdict(list)
for l in open('$OUT/realtime.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); k=('compute_n',) if 'compute_n' in d else (d['lanes'],d['busy_split'],d['defer']); b[k].append(d['ms_per_frame'])
for k,v in sorted(b.items(), key=lambda kv: min(kv[1])): print(k, min(v))"
for sc in island cave; do
for r in 1 2; do for f in 2 3 4; do for k in 4 8 16; do
  out=$(timeout -k 10 120 python3 tools/frames.py --scene $sc --batch 20 --frames 3 --factor $f --split $k 2>&1 | tail -1) || { echo "sweep failed: $out"; exit 1; }
  echo "{\"round\": $r, \"factor\": $f, \"split\": $k, \"result\": $out}"
done; done; done > $OUT/plan_$sc.jsonl
python3 -c "
import json,collections
b=collections.defaultdict(list)
for l in open('$OUT/plan_$sc.jsonl'): d=json.loads(l); b[(d['factor'],d['split'])].append(min(d['result']['ms']))
print('$sc', sorted(((round(min(v),3),k) for k,v in b.items())))"
done
