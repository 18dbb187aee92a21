#!/bin/bash
# Interleaved A/B timing of library builds on the headline workload (hrt_compute_n, 64-frame launches):
#   bash tools/ab.sh <rounds> <libA.so> <libB.so> ... [-- extra frames.py args]
# Prints one JSON line per (round, library) with ms per frame (tools/frames.py --batch $AB_BATCH, default 64).
R=$1; shift
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "$1" == "--" ] && shift
for r in $(seq 1 $R); do
  for L in "${LIBS[@]}"; do
    out=$(HRT_LIB=$L timeout -k 10 120 python3 tools/frames.py --batch ${AB_BATCH:-64} --frames 3 "$@" 2>&1 | tail -1) || { echo "{\"lib\": \"$L\", \"error\": \"$out\"}"; exit 1; }
    echo "{\"round\": $r, \"lib\": \"$L\", \"result\": $out}"
  done
done
