#!/bin/bash
# PMC passes of the bench command itself (so the profiled launch is the timed launch: one hrt_compute_n
# launch of STEPS frames after the warm-up), each pass its own rocprofv3 run (--pmc with --kernel-trace
# only).  Usage: bash tools/pmc.sh <tag> [bench.py args...]   (default: the headline, 64 frames)
# Writes gpurun_out/<tag>/summary.json and gpurun_out/<tag>/pmc_traffic.json (bench.py's roofline).
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/$TAG; mkdir -p $OUT
ARGS="--warmup 5 --steps 20 --cpu-seconds 0 --realtime-frames 0 $*"  # the driver's bench shape
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- \
    python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed: $(tail -3 $OUT/p$i.log)"; exit 1; }
done
WL=$(python3 - "$OUT/p1.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        c = json.loads(line)["config"]
        steps = json.loads(line)["steps"]
        # the timed launch's frames as the library split the steps (hrt_stats.last_frames)
        c["frames_per_launch"] = c.get("launch_frames") or min(c["frames_per_launch"], steps)
        print(" ".join(f"{k}={c[k]}" for k in ("scene", "width", "height", "spp", "bounces", "kernel_variant",
                                                 "frames_per_launch")), c["frames_per_launch"])
PY
)
FRAMES=${WL##* }; WL=${WL% *}
python3 tools/pmc_summary.py $OUT --traffic-json $OUT/pmc_traffic.json --frames $FRAMES --workload $WL > $OUT/summary.json
cat $OUT/pmc_traffic.json
