#!/bin/bash
# r04u: BVH leaf size against the current pair traversal (node pairs got dearer than triangle pairs:
# a node step tests 4 members per lane, a triangle step one packed pair).  Island (auto 2) and cave
# (auto 3), interleaved rounds, 20-frame launches.
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
for r in 1 2; do
  for L in 2 3 4 6; do
    timeout -k 10 120 python3 tools/frames.py --batch 20 --frames 3 --leaf $L > $OUT/t.log 2>&1 || { echo "island leaf $L failed"; tail -5 $OUT/t.log; exit 1; }
    echo "{\"round\": $r, \"scene\": \"island\", \"leaf\": $L, \"result\": $(tail -1 $OUT/t.log)}" >> $OUT/leaf.jsonl
  done
  for L in 3 4 6; do
    timeout -k 10 120 python3 tools/frames.py --batch 20 --frames 3 --leaf $L --scene cave --node-r 2 > $OUT/t.log 2>&1 || { echo "cave leaf $L failed"; tail -5 $OUT/t.log; exit 1; }
    echo "{\"round\": $r, \"scene\": \"cave\", \"leaf\": $L, \"result\": $(tail -1 $OUT/t.log)}" >> $OUT/leaf.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04u/leaf.jsonl"):
    d = json.loads(l); r = d["result"]
    print(d["round"], d["scene"], d["leaf"], r.get("ms_median", r.get("ms")), r.get("ms_min"))
PY
