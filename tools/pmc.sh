#!/bin/bash
# PMC passes for one kbench variant (each pass its own rocprofv3 run; --pmc never combined with traces
# other than kernel-trace).  Usage: bash tools/pmc.sh <tag> <variant> [kbench args]
set -o pipefail
TAG=$1; V=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/$TAG; mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/kbench.py --variants $V --rounds 1 "$@" > $OUT/p$i.log 2>&1 || echo "pass $i ($set) failed: $(tail -3 $OUT/p$i.log)"
done
python3 tools/pmc_summary.py $OUT
