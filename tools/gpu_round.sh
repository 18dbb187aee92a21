#!/bin/bash
# One GPU-box session: GPU tests, smoke, PMC passes of the bench command (roofline record stamped with
# this build), the bench line (N=1) and the rocprofv3 kernel-trace summary of the same bench command.
# Usage (repo root, via gpurun): bash tools/gpu_round.sh <tag> [bench.py args]
set -o pipefail
TAG=${1:-r02}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ -z "$SKIP_TESTS" ]; then  # SKIP_TESTS=1: only the PMC passes, the bench line and the kernel trace
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
fi
bash tools/pmc.sh $TAG/pmc "$@" > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc_traffic.json $OUT/pmc_traffic.json
# the bench line cites the record where it is committed (profiles/<round>/<tag>_pmc/, copied there from
# gpurun_out/<tag>/pmc_traffic.json after the call), not the scratch directory
PMC=profiles/$(echo $TAG | cut -c1-3)/${TAG}_pmc; mkdir -p $PMC
cp $OUT/pmc_traffic.json $PMC/pmc_traffic.json
timeout -k 10 600 python3 bench.py --pmc-json $PMC/pmc_traffic.json "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --pmc-json $PMC/pmc_traffic.json "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec head -4 {} \;
