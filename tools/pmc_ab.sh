#!/bin/bash
# Instruction counts of A/B library builds: one rocprofv3 --pmc pass (instruction / wait counters) of
# a 64-frame hrt_compute_n launch per build, summarised per frame by tools/pmc_ab_summary.py.
#   bash tools/pmc_ab.sh <tag> <libA.so> <libB.so> ...   -> gpurun_out/<tag>/<build>/p1, summary on stdout
#   (PMC="FETCH_SIZE" bash tools/pmc_ab.sh ...: another counter set, one rocprofv3 pass each;
#    FRAMES_ARGS="--scene cave": another workload)
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$TAG
for L in "$@"; do
  N=$(basename $(dirname $L))
  HRT_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace \
    --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY} \
    -d gpurun_out/$TAG/$N/p1 -o run --output-format csv -- python3 tools/frames.py --batch 64 --frames 1 $FRAMES_ARGS \
    > gpurun_out/$TAG/$N.log 2>&1 || { echo "pmc pass of $N failed: $(tail -3 gpurun_out/$TAG/$N.log)"; exit 1; }
done
python3 tools/pmc_ab_summary.py gpurun_out/$TAG
