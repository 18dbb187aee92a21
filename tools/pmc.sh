#!/bin/bash
# PMC passes for one kbench variant, each pass its own rocprofv3 run (--pmc with --kernel-trace only).
# Usage: bash tools/pmc.sh <tag> <variant> [--scene S --size WxH --spp N --bounces B]
# Writes gpurun_out/<tag>/summary.json and gpurun_out/<tag>/pmc_traffic.json (bench.py's `traffic`).
set -o pipefail
TAG=$1; V=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/$TAG; mkdir -p $OUT
SCENE=island; SIZE=1920x1080; SPP=64; BOUNCES=8
while [ $# -gt 0 ]; do case $1 in --scene) SCENE=$2;; --size) SIZE=$2;; --spp) SPP=$2;; --bounces) BOUNCES=$2;; esac; shift 2; done
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/kbench.py --no-ref --variants $V --rounds 1 --scene $SCENE --size $SIZE --spp $SPP --bounces $BOUNCES \
    > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed: $(tail -3 $OUT/p$i.log)"; exit 1; }
done
W=${SIZE%x*}; H=${SIZE#*x}
python3 tools/pmc_summary.py $OUT --traffic-json $OUT/pmc_traffic.json \
  --workload scene=$SCENE width=$W height=$H spp=$SPP bounces=$BOUNCES variant=$V > $OUT/summary.json
cat $OUT/pmc_traffic.json
