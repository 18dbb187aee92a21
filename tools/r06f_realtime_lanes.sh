set -o pipefail
mkdir -p gpurun_out/r06f
for q in 4 8; do
 for L in 4 6; do
  GPU_MAX_HW_QUEUES=$q HRT_LIB=epq_raytracer_amd/build/ab_lanes$L/libhip_raytrace.so timeout -k 10 200 python3 tools/realtime.py --lanes 3 $L --busy-split 2 3 --defer 0 --rounds 1 > gpurun_out/r06f/rt_q${q}_l$L.jsonl 2>&1 || { echo fail; tail -3 gpurun_out/r06f/rt_q${q}_l$L.jsonl; exit 1; }
  echo "q=$q L=$L"; cat gpurun_out/r06f/rt_q${q}_l$L.jsonl | cut -c1-200
 done
done
