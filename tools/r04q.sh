# Realtime loop (per-frame traces) against the planner's split knobs: single lane (a frame alone) and
# three lanes with half grids.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 400 python3 tools/realtime.py --lanes 1 3 --busy-split 2 --defer 0 --split 0 16 64 --factor -1 1 4 \
  --rounds 2 --frames 32 > $O/rt_split.jsonl 2> $O/rt_split.err
