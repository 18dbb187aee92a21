#!/bin/bash
# One GPU-box session: smoke, bench (N=1), rocprofv3 kernel-trace summary of the same bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/$TAG/smoke.log; exit 1; }
timeout -k 10 600 python3 bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 "$@" > gpurun_out/$TAG/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/$TAG/prof.log; exit 1; }
find gpurun_out/$TAG/prof -name '*kernel_stats.csv' -exec cat {} \;
