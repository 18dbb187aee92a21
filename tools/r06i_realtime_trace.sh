#!/bin/bash
# The realtime loop's host floor (a 64x64 frame) and a kernel trace of the 1080p loop (3 lanes, busy split 2).
set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python3 tools/realtime.py --size 64x64 --lanes 1 3 --busy-split 2 --defer 0 --rounds 1 > $OUT/small.jsonl 2>&1 || { echo small failed; tail -3 $OUT/small.jsonl; exit 1; }
cat $OUT/small.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python3 tools/realtime.py --lanes 3 --busy-split 2 --defer 0 --rounds 1 > $OUT/kt.log 2>&1 || { echo kt failed; tail -5 $OUT/kt.log; exit 1; }
grep ms_per $OUT/kt.log
