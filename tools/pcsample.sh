#!/bin/bash
# PC sampling of the bench command's trace kernel (rocprofv3, stochastic sampling on gfx950): which
# instructions the waves sit at, with their stall reasons.  Usage (via gpurun): bash tools/pcsample.sh <tag> [bench args]
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 -L > $OUT/list.txt 2>&1 || echo "list rc=$?"
grep -i -A30 "pc sampl\|PC_SAMPL\|pc-sampl" $OUT/list.txt | head -60
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} \
  --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-65536} \
  -d $OUT/pcs -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --realtime-frames 0 "$@" \
  > $OUT/pcs.log 2>&1
rc=$?
echo "pcs rc=$rc"; tail -5 $OUT/pcs.log
find $OUT/pcs -type f | head
