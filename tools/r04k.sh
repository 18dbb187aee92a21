#!/bin/bash
# r04k: instruction-cache and scalar-cache counters of the product build (the bench's timed launch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r04k; mkdir -p $OUT
ARGS="--warmup 5 --steps 20 --cpu-seconds 0 --realtime-frames 0"
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU" "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed: $(tail -3 $OUT/p$i.log)"; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for p in sorted(glob.glob(out + "/p*")):
    per = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for f in glob.glob(p + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_bundle_wq<false>" not in r["Kernel_Name"]: continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if per:
        d = max(per.values(), key=lambda c: sum(c.values()))
        print(p.split("/")[-1], {k: int(v) for k, v in d.items()})
PY
