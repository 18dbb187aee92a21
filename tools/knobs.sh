#!/bin/bash
# Interleaved sweep of runtime options on the production library (tools/frames.py, 64-frame launches):
#   bash tools/knobs.sh <rounds> <scene> "<frames.py args A>" "<args B>" ...
R=$1; SCENE=$2; shift 2
for r in $(seq 1 $R); do
  for A in "$@"; do
    out=$(timeout -k 10 150 python3 tools/frames.py --batch 64 --frames 3 --scene $SCENE $A 2>&1 | tail -1) || { echo "{\"args\": \"$A\", \"error\": \"$out\"}"; exit 1; }
    echo "{\"round\": $r, \"args\": \"$A\", \"result\": $out}"
  done
done
