#!/bin/bash
# r04ab: bounce-batch threshold (HRT_OPT_SECONDARY_BATCH; 0 = auto) on the final build, island and cave.
set -o pipefail
OUT=gpurun_out/r04ab; mkdir -p $OUT
for r in 1 2; do
  for S in 0 16 24 32 48; do
    timeout -k 10 120 python3 tools/frames.py --batch 20 --frames 3 --sec-batch $S > $OUT/t.log 2>&1 || { echo "island $S failed"; tail -5 $OUT/t.log; exit 1; }
    echo "{\"round\": $r, \"scene\": \"island\", \"sec_batch\": $S, \"result\": $(tail -1 $OUT/t.log)}" >> $OUT/sec.jsonl
    timeout -k 10 120 python3 tools/frames.py --batch 20 --frames 3 --sec-batch $S --scene cave --node-r 2 > $OUT/t.log 2>&1 || { echo "cave $S failed"; tail -5 $OUT/t.log; exit 1; }
    echo "{\"round\": $r, \"scene\": \"cave\", \"sec_batch\": $S, \"result\": $(tail -1 $OUT/t.log)}" >> $OUT/sec.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04ab/sec.jsonl"):
    d = json.loads(l); r = d["result"]
    print(d["round"], d["scene"], d["sec_batch"], r.get("ms_median", r.get("ms")))
PY
