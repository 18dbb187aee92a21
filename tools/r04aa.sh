#!/bin/bash
# r04aa: the realtime loop (per-frame traces) on the final build: lanes 3 with busy split 2 / 3, planner
# factor auto / 4, split auto / 16.
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 400 python3 tools/realtime.py --lanes 3 --busy-split 2 3 --defer 0 --split 0 16 --factor -1 4 \
  --rounds 2 --frames 32 > $O/rt.jsonl 2> $O/rt.err || { echo "realtime failed"; tail -5 $O/rt.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r04aa/rt.jsonl"):
    d = json.loads(l)
    print(d.get("lanes"), d.get("busy_split"), d.get("split"), d.get("factor"), d.get("compute_n"), d["ms_per_frame"])
PY
