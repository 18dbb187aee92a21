#!/bin/bash
# r03ag: runtime-knob re-check on the current build after the r03 traversal changes (node radius mode,
# leaf size, group width) on cave and island.
set -o pipefail
OUT=gpurun_out/r03ag; mkdir -p $OUT
timeout -k 10 900 bash tools/knobs.sh 2 cave "" "--node-r 1" "--node-r 2" "--leaf 3" "--leaf 4" "--width 3" > $OUT/knobs_cave.jsonl 2>&1 || { echo "cave knobs failed"; tail -5 $OUT/knobs_cave.jsonl; exit 1; }
timeout -k 10 900 bash tools/knobs.sh 2 island "" "--node-r 2" "--leaf 1" "--leaf 3" "--width 3" > $OUT/knobs_island.jsonl 2>&1 || { echo "island knobs failed"; tail -5 $OUT/knobs_island.jsonl; exit 1; }
for S in cave island; do python3 -c "
import json
for l in open('$OUT/knobs_$S.jsonl'):
    d=json.loads(l); print('$S', d['round'], repr(d['args']), min(d['result']['ms']) if 'result' in d else d)
"; done
